# Round 5: narrowphase of the divergent ScratchItch pool-27 pair, the dressing parity tests and smoke.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5
TASK=1 K=27 SA=50 SB=165 timeout -k 10 300 python3 -u tools/dbg_np_state.py > gpurun_out/r5/np27.log 2>&1 || exit 11
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_dressing.py > gpurun_out/r5/t2_dress.log 2>&1 || exit 12
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/smoke.log 2>&1 || exit 13
timeout -k 10 300 python3 bench.py --task DressingJaco-v0 --facade --steps 600 > gpurun_out/r5/facade_dress.json 2> gpurun_out/r5/facade_dress.err || exit 14
