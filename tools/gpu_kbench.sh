cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && mkdir -p gpurun_out
LATTICEUM_AMD_NTT=stockham timeout -k 10 200 python tools/kbench.py > gpurun_out/kb_stockham.json 2>gpurun_out/kb_err1.log && \
LATTICEUM_AMD_NTT=wave timeout -k 10 200 python tools/kbench.py > gpurun_out/kb_wave.json 2>gpurun_out/kb_err2.log
cat gpurun_out/kb_stockham.json gpurun_out/kb_wave.json
