# One GPU call: parity suite, smoke, bench line, flake probe (each step time-limited, chained with &&).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r/smoke.log 2>&1 && \
timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --cpu-seconds 10 > gpurun_out/r/bench.json 2> gpurun_out/r/bench.err && \
timeout -k 10 300 python3 tools/flake.py 4096 12 > gpurun_out/r/flake.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r/pytest_gpu.log | tail -8
tail -2 gpurun_out/r/smoke.log
tail -c 1500 gpurun_out/r/bench.json
grep -v amdgpu gpurun_out/r/flake.log | tail -8
echo rc=$rc
