# Round check: parity suite + smoke, then the round profile (kernel-trace stats, PMC passes, full bench line).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/fin
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/fin/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin/smoke.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/fin/pytest_gpu.log | tail -6
tail -1 gpurun_out/fin/smoke.log
if [ $rc -ne 0 ]; then echo rc=$rc; exit $rc; fi
bash tools/gpu_profile.sh
