# Round-5 evidence, part 2: full bench lines (with the CPU baseline) of the four tasks, the policy-
# evaluation harness, and the facade benches (AVRTorchVecEnv with rollovers).  Output: gpurun_out/g5/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/g5
timeout -k 10 300 python3 bench.py > gpurun_out/g5/bench_feeding.json 2> gpurun_out/g5/b0.err || exit 13
timeout -k 10 300 python3 bench.py --task ScratchItchPR2-v0 > gpurun_out/g5/bench_scratch.json 2> gpurun_out/g5/b1.err || exit 14
timeout -k 10 300 python3 bench.py --task BedBathingPR2-v0 > gpurun_out/g5/bench_bedbath.json 2> gpurun_out/g5/b2.err || exit 15
timeout -k 10 300 python3 bench.py --task DressingJaco-v0 > gpurun_out/g5/bench_dressing.json 2> gpurun_out/g5/b3.err || exit 16
timeout -k 10 300 python3 bench.py --policy-eval > gpurun_out/g5/policy_eval.json 2> gpurun_out/g5/pe.err || exit 17
for T in FeedingJaco-v0 ScratchItchPR2-v0 BedBathingPR2-v0 DressingJaco-v0; do
  timeout -k 10 300 python3 bench.py --task $T --facade --steps 600 > gpurun_out/g5/facade_$T.json 2> gpurun_out/g5/facade_$T.err || exit 18
done
for f in gpurun_out/g5/bench_*.json gpurun_out/g5/facade_*.json gpurun_out/g5/policy_eval.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[1], round(d['value']), d.get('unit'))" $f
done
