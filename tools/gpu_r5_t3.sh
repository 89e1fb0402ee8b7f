# Round 5: the reworked parity tests (PR2 launch shape with the 16-member fp32 ensemble, contact
# statistics against the fp32 and fp64 oracles, BedBathing 200 steps, the wheelchair drift against
# an fp32 ensemble), then the chain-latency profile (tools/gpu_r5_prof.sh).  Output: gpurun_out/r5t3/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t3
timeout -k 10 700 python3 -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu tests/test_pr2_launch_shape.py \
  "tests/test_bedbath.py::test_bedbath_200_steps_within_1e3" "tests/test_gpu_parity.py::test_coop_capped_env_drift_vs_oracle" > gpurun_out/r5t3/tests.log 2>&1
rc=$?
echo tests rc=$rc
case $rc in 124|134|137|139) exit $rc ;; esac
bash tools/gpu_r5_prof.sh
