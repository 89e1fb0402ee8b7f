set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --cpu-seconds 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"
tail -c 3000 gpurun_out/bench1.json
tail -5 gpurun_out/bench1.err
