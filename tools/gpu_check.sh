# GPU test suite + kernel-trace stats of a short bench (per-kernel split)
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/chk
timeout -k 10 600 python3 -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/chk/pytest_gpu.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/chk/kt -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/chk/kt_bench.log 2>&1
rc=$?
tail -3 gpurun_out/chk/pytest_gpu.log
grep -v amdgpu.ids gpurun_out/chk/kt_bench.log | grep '"value"' | cut -c1-200
echo rc=$rc
