#!/bin/bash
# bench.py's N = 2 control flow on a one-GPU box: two ranks on cuda:0 over gloo
# (LATTICEUM_AMD_REHEARSE_ONE_GPU); the sharded fold's RCCL communicator
# cannot form on one GPU and reports its error (or the watchdog's timeout)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LATTICEUM_AMD_REHEARSE_ONE_GPU=1
mkdir -p gpurun_out
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --w 2048 --no-cpu-baseline \
  --detail gpurun_out/rehearse2_detail.json \
  > gpurun_out/rehearse2.log 2>&1
rc=$?; echo "rc=$rc"; grep -v '^{' gpurun_out/rehearse2.log | tail -20
python3 -c "
import json; L=[l for l in open('gpurun_out/rehearse2.log') if l.startswith('{')]; print(len(L), 'json lines')
print('last line bytes', len(L[-1]))
d=json.loads(L[-1]); print(d['n_gpus'], round(d['value'],2), d.get('sharded_fold'), 'detail', d.get('detail'))
for k, v in (d.get('side') or {}).items(): print(k, v)
full=json.load(open(d['detail'])); print('detail keys', sorted(full)[:12])"
exit $rc
