"""Synthetic scenes for the oracle's dynamics known-answer tests: a fixed-base chain of revolute
links built with the model compiler's Scene (no shapes, so no contacts), plus one far-away free
sphere (the weld constraint of the FeedingJaco glue needs a child body; its max force is set to 0,
so the weld never acts)."""
import numpy as np

from avr import _abi as ABI
from avr import model_compiler as MC


def chain_scene(links, free_inertia=(4e-5, 4e-5, 4e-5), free_mass=1.0):
    """links: dicts with parent (-1 = fixed base), axis, jpos (in the parent link frame), com_pos,
    mass, inertia (principal, COM frame = link frame orientation)."""
    S = MC.Scene()
    rob = dict(name=[], parent=[], jtype=[], dof=[], jpos=[], jquat=[], axis=[], com_pos=[], com_quat=[], mass=[],
               inertia=[], lower=[], upper=[], has_limit=[], shapes=[], friction=[])
    for i, L in enumerate(links):
        rob['name'].append('l%d' % i)
        rob['parent'].append(L['parent'])
        rob['jtype'].append(MC.J_REVOLUTE)
        rob['dof'].append(i)
        rob['jpos'].append(np.asarray(L['jpos'], float))
        rob['jquat'].append(np.array([0, 0, 0, 1.0]))
        ax = np.asarray(L['axis'], float)
        rob['axis'].append(ax / np.linalg.norm(ax))
        rob['com_pos'].append(np.asarray(L['com_pos'], float))
        rob['com_quat'].append(np.array([0, 0, 0, 1.0]))
        rob['mass'].append(float(L['mass']))
        rob['inertia'].append(np.asarray(L['inertia'], float))
        rob['lower'].append(0.0)
        rob['upper'].append(-1.0)
        rob['has_limit'].append(0)
        rob['shapes'].append([])
        rob['friction'].append(0.5)
    rob['ndof'] = len(links)
    S.robot = rob
    S.robot_base_pos = np.zeros(3)
    S.robot_base_quat = np.array([0, 0, 0, 1.0])
    S.free = [dict(name='probe', mass=free_mass, inertia=np.asarray(free_inertia, float), gravity=np.zeros(3))]
    fb = S.add_body(MC.KIND_FREE, 0, [MC.Shape(MC.SPHERE, radius=0.01)], 0.5, 'probe', single=True)
    S.static = []
    S.pairs = []
    A = MC.to_arrays(S)
    A['human_slot_link'] = np.zeros(0, np.int32)
    A['n_pairs_base'] = np.int32(0)
    A['task_arm_dofs'] = np.arange(len(links), dtype=np.int32)[:7]
    A['task_finger_dofs'] = np.zeros(0, np.int32)
    A['task_tool_link'] = np.int32(0)
    A['task_torso_link'] = np.int32(0)
    A['task_tool_offset'] = np.array([0, 0, 0, 0, 0, 0, 1.0])
    A['task_head_link'] = np.int32(0)
    A['task_mouth_male'] = np.zeros(3)
    A['task_mouth_female'] = np.zeros(3)
    for k in ('task_spoon_body', 'task_bowl_body', 'task_food_body0', 'task_table_body'):
        A[k] = np.int32(fb)
    A['task_human_body0'] = np.int32(0)
    A['task_head_slot'] = np.int32(0)
    return A


def desc(A, **params):
    """ModelDesc with no damping, no weld force and the given overrides (e.g. robot_gravity)."""
    P = dict(linear_damping=0.0, angular_damping=0.0, fixed_max_force=0.0, default_motor_impulse=0.0)
    P.update(params)
    return ABI.ModelDesc(A, P)


def state(md, q, qd=None, kp=None, target=None, maximp=None):
    """One env's state: joint values, motors (kp 0 + impulse 0 = motors off), probe far away."""
    st = np.zeros(ABI.STATE_WORDS)
    n = len(q)
    st[ABI.S_Q:ABI.S_Q + n] = q
    if qd is not None:
        st[ABI.S_QD:ABI.S_QD + n] = qd
    st[ABI.S_KP:ABI.S_KP + n] = 0.0 if kp is None else kp
    st[ABI.S_QTGT:ABI.S_QTGT + n] = 0.0 if target is None else target
    st[ABI.S_MAXIMP:ABI.S_MAXIMP + n] = 0.0 if maximp is None else maximp
    f = ABI.S_FREE
    st[f:f + 3] = [100.0, 100.0, 100.0]
    st[f + 3:f + 7] = [0, 0, 0, 1]
    return st[None]
