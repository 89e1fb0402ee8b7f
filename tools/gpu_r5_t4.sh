# Round 5: the PR2 launch-shape tests (bookkeeping against the ensemble), then how much of kernel
# a's launch the EPA / cooperative pairs cost: interleaved benches of the shipped build and a
# diagnostic build that never runs one (AVR_COOP_CAP=0), and the per-wave timeline of the latter.
# Output: gpurun_out/r5t4/, gpurun_out/ab/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t4
timeout -k 10 500 python3 -u -m pytest -v -s --timeout 450 --timeout-method thread -m gpu tests/test_pr2_launch_shape.py -k launch_shape > gpurun_out/r5t4/tests.log 2>&1
rc=$?
echo tests rc=$rc
case $rc in 124|134|137|139) exit $rc ;; esac
VARIANTS="default noepa" ROUNDS=2 bash tools/gpu_ab_variants.sh || exit 12
timeout -k 10 200 python3 tools/wavetime.py 1024 /root/repo/_ab/libavr_noepawt.so > gpurun_out/r5t4/wt1k_noepa.log 2>&1 || exit 13
