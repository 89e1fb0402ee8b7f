# Round 5: the reworked parity tests (PR2 launch shape with contact picks and the rounding ensemble,
# contact statistics at 512 envs, the EPA-budget drift against the fp32 ensemble, the reference-format
# recording replay).  Output: gpurun_out/r5/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_pr2_launch_shape.py tests/test_record_eval.py \
  "tests/test_gpu_parity.py::test_coop_capped_env_drift_vs_oracle" > gpurun_out/r5/t1.log 2>&1
