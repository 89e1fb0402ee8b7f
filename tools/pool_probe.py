"""Dump the bench's reset pool of a task (the PR2 tasks' pools come from the device base-pose
search) to an .npy file for offline analysis with the oracle.
   python tools/pool_probe.py <task-name> <out.npy>"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'assistive-vr-gym_amd'))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from avr import _abi as ABI  # noqa: E402

name, out = sys.argv[1], sys.argv[2]
T = bench.TASKS[name]
A = ABI.load_scene(T['task'])
md = ABI.ModelDesc(A)
S, meta = bench.reset_pool(T['task'], A, md, list(range(T['pool'])), 'random')
np.save(out, S.astype(np.float32))
print(name, S.shape)
