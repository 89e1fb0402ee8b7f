set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ab gpurun_out/fp
TASKS=none bash tools/gpu_ab4.sh > gpurun_out/ab/fp.txt 2>&1; cat gpurun_out/ab/fp.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "coop_cap or graph" tests/test_scratch.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_new.log 2>&1 || exit 12
timeout -k 10 400 python3 tools/facade_flag_probe.py > gpurun_out/fp/flag2.txt 2>&1 || exit 13
TASK=FeedingJaco-v0 VARIANTS="default fab" bash tools/gpu_variants.sh > gpurun_out/ab/var_fab_f.txt 2>&1 || exit 14
TASK=ScratchItchPR2-v0 VARIANTS="default fab" bash tools/gpu_variants.sh > gpurun_out/ab/var_fab_s.txt 2>&1 || exit 15
