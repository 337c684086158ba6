#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/exp/enqueue_probe.hip -o /tmp/eq_probe 2>/dev/null && timeout -k 10 60 /tmp/eq_probe
