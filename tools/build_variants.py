"""Experiment builds of libavr.so: _ab/libavr_<name>.so (VARDIR overrides) with the extra hipcc
flags of VARIANTS (tools/gpu_ab_variants.sh benches them against the shipped build).

    python tools/build_variants.py name [name ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
from avr import build as B  # noqa: E402

VARIANTS = {
    # round 1 flag experiments
    'ftz': ('-fgpu-flush-denormals-to-zero',),
    'ftzapx': ('-fgpu-flush-denormals-to-zero', '-fgpu-approx-transcendentals'),
    'slp': ('-fslp-vectorize',),
    'unclustered': ('-mllvm', '-amdgpu-disable-unclustered-high-rp-reschedule'),
    # round 2
    'fdiv': ('-fno-hip-fp32-correctly-rounded-divide-sqrt',),
    'dc1': ('-DB4_DC=1',), 'dc3': ('-DB4_DC=3',), 'dc4': ('-DB4_DC=4',),
    'dn2': ('-DB4_DN=2',), 'dn3': ('-DB4_DN=3',), 'dn4': ('-DB4_DN=4',), 'dc2': ('-DB4_DC=2',),
    'np4': ('-DNP_WAVES=4',), 'ne1': ('-DNP_ENVS=1',), 'ne2': ('-DNP_ENVS=2',), 'ne8': ('-DNP_ENVS=8',),
    'l11k': ('-DB4_LDSW=11264',), 'l12k': ('-DB4_LDSW=12288',), 'aw4': ('-DAVR_WAVES_PER_EU=4',), 'aw3': ('-DAVR_WAVES_PER_EU=3',),
    # round 3
    'nopk': ('-DB4_PK=0',), 'slp3': ('-fslp-vectorize',),
    'l8k': ('-DB4_LDSW=8192',), 'l7k': ('-DB4_LDSW=7168',), 'l6k': ('-DB4_LDSW=6144',), 'np4nb4': ('-DNP_WAVES=4', '-DGJK_NB=4'),
    'coopk': ('-DAVR_COOP_KERNEL=1',), 'ml': ('-DAVR_MINV_LAUNDER=1',), 'mlc': ('-DAVR_MINV_LAUNDER=1', '-DAVR_COOP_KERNEL=1'),
    'mlc2': ('-DAVR_MINV_LAUNDER=1', '-DAVR_COOP_KERNEL=1', '-DAVR_WAVES_PER_EU=2'),
    'nofp': ('-DB4_FPAIR=0',),
    # round 5
    'noepa': ('-DAVR_COOP_CAP=0', '-DAVR_COOP_PERSIST=0'),     # diagnostic only: no EPA / cooperative pair ever runs
    'noepawt': ('-DAVR_COOP_CAP=0', '-DAVR_COOP_PERSIST=0', '-DAVR_WAVETIME'),
    'coopk5': ('-DAVR_COOP_KERNEL=1',), 'np5': ('-DNP_WAVES=5',), 'dc2r5': ('-DB4_DC=2',),
    # round 6: the AMDGPU machine scheduler's strategies
    'mclause': ('-mllvm', '-amdgpu-sched-strategy=max-memory-clause'), 'ilp': ('-mllvm', '-amdgpu-sched-strategy=max-ilp'),
    'itilp': ('-mllvm', '-amdgpu-sched-strategy=iterative-ilp'),
    'nonl': ('-DB4_NC_LDS=0',), 'fnl': ('-DB4_NC_LDS=1',), 'fnl12': ('-DB4_NC_LDS=1', '-DB4_LDSW=12288'), 'fnl11': ('-DB4_NC_LDS=1', '-DB4_LDSW=11264'), 'dnl2': ('-DB4_DNL=2',), 'noml': ('-DAVR_MINV_LAUNDER=0',),
    'cr0': ('-DAVR_COOP_ROWS=0',), 'ccheck': ('-DAVR_COOP_CHECK',), 'cr2': ('-DAVR_COOP_ROWS=2',), 'cr8': ('-DAVR_COOP_ROWS=8',),
}


OUT = os.environ.get('VARDIR', os.path.join(ROOT, '_ab'))    # _ab/: git-ignored, travels with gpurun


def main(names):
    os.makedirs(OUT, exist_ok=True)
    for n in names:
        out = os.path.join(OUT, 'libavr_%s.so' % n)
        B.build_lib(extra=VARIANTS[n], out=out)
        print(out)


if __name__ == '__main__':
    main(sys.argv[1:] or sorted(VARIANTS))
