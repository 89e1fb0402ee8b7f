# Round-5 evidence, part 3: the whole GPU suite and smoke() on the final tree.  Output: gpurun_out/g5f/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/g5f
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/g5f/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; tail -3 gpurun_out/g5f/pytest.log
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g5f/smoke.log 2>&1
echo smoke rc=$?; tail -5 gpurun_out/g5f/smoke.log
