# Round 5: contact pools after one sub-step (GPU vs fp32 / fp64 oracles) for the FeedingJaco
# arm-in-wheelchair state and the ScratchItch launch-shape pool state 27, and the narrowphase of
# state 27's suspect pair.  Output: gpurun_out/r5p/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5p
TASK=0 timeout -k 10 200 python3 -u tools/dbg_pool_diff.py > gpurun_out/r5p/pool_wheel.log 2>&1 || exit 11
TASK=1 K=27 timeout -k 10 200 python3 -u tools/dbg_pool_diff.py > gpurun_out/r5p/pool_s27.log 2>&1 || exit 12
TASK=1 K=27 NSUB=5 timeout -k 10 200 python3 -u tools/dbg_pool_diff.py > gpurun_out/r5p/pool_s27_5.log 2>&1 || exit 13
TASK=1 K=27 SA=50 SB=165 timeout -k 10 300 python3 -u tools/dbg_np_state.py > gpurun_out/r5p/np27.log 2>&1 || exit 14
