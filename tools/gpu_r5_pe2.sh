# Round 5: the policy-evaluation harness twice, after evaluate() gained one untimed policy forward
# before its timed loop (first-process cost check).  Output: gpurun_out/g5/pe2_*.json
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/g5
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --policy-eval > gpurun_out/g5/pe2_$r.json 2> gpurun_out/g5/pe2_$r.err || exit 17
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(round(d['value']), d['ms_per_step'])" gpurun_out/g5/pe2_$r.json
done
timeout -k 10 300 python3 -u -m pytest tests -m gpu -k 'policy' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/g5/pe2_tests.log 2>&1; echo "policy tests rc=$?"; tail -1 gpurun_out/g5/pe2_tests.log
nproc; uptime
