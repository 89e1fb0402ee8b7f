# Round 5 baseline on the restored tree: GPU suite, smoke, the FeedingJaco bench line and a kernel trace.
# Output: gpurun_out/r5b/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5b
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r5b/pytest.log 2>&1
rc=$?
echo pytest rc=$rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5b/smoke.log 2>&1 || exit 12
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5b/bench_feeding.json 2> gpurun_out/r5b/b0.err || exit 13
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5b/kt -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r5b/kt.log 2>&1 || exit 14
find gpurun_out/r5b/kt -name '*stats*' -exec cp {} gpurun_out/r5b/ \;
rm -rf gpurun_out/r5b/kt
exit $rc
