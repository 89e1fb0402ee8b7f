# GPU test suite (parity through the C-ABI) + determinism probe
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/t
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python3 tools/dbg4.py 64 > gpurun_out/t/det.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/t/pytest_gpu.log | tail -20
grep -v amdgpu gpurun_out/t/det.log | tail -2 | cut -c1-200
echo rc=$rc
