# Round 5: the policy-evaluation harness twice more (host-bound loop: box-to-box variance check).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/g5
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --policy-eval > gpurun_out/g5/policy_eval_$r.json 2> gpurun_out/g5/pe_$r.err || exit 17
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(round(d['value']), d['ms_per_step'])" gpurun_out/g5/policy_eval_$r.json
done
nproc; uptime
