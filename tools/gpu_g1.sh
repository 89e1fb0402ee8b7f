set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/g1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/g1/bench.json 2> gpurun_out/g1/bench.err && \
timeout -k 10 300 python3 tools/prof_phases.py 4096 > gpurun_out/g1/prof_phases.txt 2>&1
rc=$?
tail -c 1200 gpurun_out/g1/bench.json
grep -v amdgpu.ids gpurun_out/g1/prof_phases.txt | tail -28
echo rc=$rc
