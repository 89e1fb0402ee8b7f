# Round-end evidence: GPU suite, smoke, full bench lines (with the CPU baseline) and facade benches
# (AVRTorchVecEnv with rollovers) for the four tasks, the policy-eval harness and fresh-action facade.  Output: $O/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && O=gpurun_out/${OUT:-g1} && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 11
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 12
timeout -k 10 300 python3 bench.py > $O/bench_feeding.json 2> $O/b0.err || exit 13
timeout -k 10 300 python3 bench.py --task ScratchItchPR2-v0 > $O/bench_scratch.json 2> $O/b1.err || exit 14
timeout -k 10 300 python3 bench.py --task BedBathingPR2-v0 > $O/bench_bedbath.json 2> $O/b2.err || exit 15
timeout -k 10 300 python3 bench.py --task DressingJaco-v0 > $O/bench_dressing.json 2> $O/b3.err || exit 15
timeout -k 10 300 python3 bench.py --policy-eval > $O/policy_eval.json 2> $O/pe.err || exit 17
timeout -k 10 300 python3 bench.py --facade --fresh-actions --steps 600 > $O/facade_fresh.json 2> $O/ff.err || exit 18
for T in FeedingJaco-v0 ScratchItchPR2-v0 BedBathingPR2-v0 DressingJaco-v0; do
  timeout -k 10 300 python3 bench.py --task $T --facade --steps 600 > $O/facade_$T.json 2> $O/facade_$T.err || exit 16
done
