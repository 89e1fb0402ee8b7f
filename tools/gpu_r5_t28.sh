# Round 5: GPU narrowphase results on the FeedingJaco near-contact queries (offline diagnosis).
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t28
timeout -k 10 200 python3 tools/dump_np_near.py 0 gpurun_out/r5t28/np0.npz
