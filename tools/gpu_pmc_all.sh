# PMC passes (25-step window) + kernel traces for all three tasks, then the facade bench probe.
set -o pipefail
cd /root/repo
bash tools/gpu_profile_all.sh || exit 11
mkdir -p gpurun_out/fp && timeout -k 10 300 python3 bench.py --facade --steps 600 > gpurun_out/fp/fb.json 2>/dev/null || exit 12
