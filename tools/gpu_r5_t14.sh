# Round 5: the reset IK / self-contact tests after the cooperative resolution of handed-on
# self-contact pairs, and smoke().  Output: gpurun_out/r5t14/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t14
timeout -k 10 600 python3 -u -m pytest -v -s --timeout 500 --timeout-method thread -m gpu tests/test_reset_ik.py tests/test_dressing.py > gpurun_out/r5t14/tests.log 2>&1
rc=$?; echo tests rc=$rc; case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5t14/smoke.log 2>&1
rc=$?; echo smoke rc=$rc
