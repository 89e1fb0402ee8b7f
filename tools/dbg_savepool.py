"""Save the launch-shape pools (device-settled BedBathing arms) for host-side analysis."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'assistive-vr-gym_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'tests'))
import test_pr2_launch_shape as T
os.makedirs('gpurun_out/pool', exist_ok=True)
for task in (1, 2):
    A, md, L, P, isc = T._pool(task, 16)
    np.save('gpurun_out/pool/P%d.npy' % task, P)
    print(task, P.shape, flush=True)
