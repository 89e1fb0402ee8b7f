"""ctypes mirror of include/avr_model.h (`avr_model_desc`) plus the state-block offsets, and
`build_desc()` which turns a compiled scene (`avr/data/*.npz`) into a descriptor.

The descriptor only holds pointers; `ModelDesc` keeps the numpy arrays alive.
"""
import ctypes as C
import os

import numpy as np

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data')

# ---- capacities / offsets (must match include/avr_model.h) ----
ABI_VERSION = 6
TASK_FEEDING, TASK_SCRATCH, TASK_BEDBATH, TASK_DRESSING = 0, 1, 2, 3
DESC_HC = 8                               # avr_model_desc hc_* capacity
BODY_ROBOT, BODY_FREE, BODY_STATIC, BODY_HUMAN, BODY_RSTATIC = 0, 1, 2, 3, 4
# FeedingJaco-v0 layout (module-level names; the ScratchItchPR2-v0 layout is `SI` below)
MAX_LINKS, MAX_DOF, MAX_FREE, MAX_HUMAN, MAX_CONTACTS, HC_N = 20, 14, 10, 20, 96, 4
MAX_FOOD, ACT_DIM, OBS_DIM, INFO_DIM = 8, 7, 25, 2
FB_WORDS, CP_WORDS = 13, 16
S_Q = 0
S_QD = S_Q + MAX_DOF
S_QTGT = S_QD + MAX_DOF
S_KP = S_QTGT + MAX_DOF
S_MAXIMP = S_KP + MAX_DOF
S_FREE = S_MAXIMP + MAX_DOF
S_TASK = S_FREE + MAX_FREE * FB_WORDS
T_TARGET, T_ITER, T_SUCCESS, T_ALIVE, T_HIT, T_GENDER, T_FLAGS, T_NCP, T_HDYN, T_WORDS = 0, 3, 4, 5, 6, 7, 8, 9, 10, 16
T_COOPN = 15        # consecutive sub-steps with more than 4 EPAs (the kernels' EPA cap; all tasks)
S_HUMAN = S_TASK + T_WORDS
S_HCH = S_HUMAN + MAX_HUMAN * 7          # [HC_N] target_human_joint_positions, [HC_N] human_tremors
S_CP = S_HCH + 2 * HC_N
STATE_WORDS = S_CP + MAX_CONTACTS * CP_WORDS
CP_SA, CP_SB, CP_LA, CP_LB, CP_N, CP_DIST, CP_IMP, CP_LIFE, CP_PAIR = 0, 1, 2, 5, 8, 11, 12, 13, 14


class _Layout:
    """State layout of one task (include/avr_model.h), attribute names as the module-level ones."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


FEEDING = _Layout(TASK=TASK_FEEDING, MAX_LINKS=MAX_LINKS, MAX_DOF=MAX_DOF, MAX_FREE=MAX_FREE, MAX_HUMAN=MAX_HUMAN,
                  MAX_CONTACTS=MAX_CONTACTS, HC_N=HC_N, ACT_DIM=ACT_DIM, OBS_DIM=OBS_DIM, INFO_DIM=INFO_DIM,
                  S_Q=S_Q, S_QD=S_QD, S_QTGT=S_QTGT, S_KP=S_KP, S_MAXIMP=S_MAXIMP, S_FREE=S_FREE, S_TASK=S_TASK,
                  T_TARGET=T_TARGET, T_ITER=T_ITER, T_SUCCESS=T_SUCCESS, T_ALIVE=T_ALIVE, T_HIT=T_HIT, T_GENDER=T_GENDER,
                  T_FLAGS=T_FLAGS, T_NCP=T_NCP, T_HDYN=T_HDYN, T_COOPN=T_COOPN, T_WORDS=T_WORDS, S_HUMAN=S_HUMAN, S_HCH=S_HCH, S_CP=S_CP,
                  STATE_WORDS=STATE_WORDS)


def _scratch_layout(task=TASK_SCRATCH):
    L = dict(TASK=task, MAX_LINKS=32, MAX_DOF=24, HC_N=8, MAX_FREE=1, MAX_HUMAN=20, MAX_CONTACTS=64,
             ACT_DIM=7, OBS_DIM=30 if task == TASK_SCRATCH else 24, INFO_DIM=2)
    L['S_Q'] = 0
    L['S_QD'] = L['S_Q'] + L['MAX_DOF']
    L['S_QTGT'] = L['S_QD'] + L['MAX_DOF']
    L['S_KP'] = L['S_QTGT'] + L['MAX_DOF']
    L['S_MAXIMP'] = L['S_KP'] + L['MAX_DOF']
    L['S_FREE'] = L['S_MAXIMP'] + L['MAX_DOF']
    L['S_RBASE'] = L['S_FREE'] + L['MAX_FREE'] * FB_WORDS
    L['S_TASK'] = L['S_RBASE'] + 8
    L.update(T_TARGET=0, T_ITER=3, T_SUCCESS=4, T_LIMB=5, T_STRENGTH=6, T_GENDER=7, T_FLAGS=8, T_NCP=9, T_HDYN=10,
             T_PREV=11, T_TREMOR=14, T_COOPN=15, T_ONARM=16, T_WORDS=24)
    L['S_HUMAN'] = L['S_TASK'] + L['T_WORDS']
    L['S_HCH'] = L['S_HUMAN'] + L['MAX_HUMAN'] * 7      # [HC_N] targets, tremors, lower, upper limits
    L['S_CP'] = L['S_HCH'] + 4 * L['HC_N']
    L['STATE_WORDS'] = L['S_CP'] + L['MAX_CONTACTS'] * CP_WORDS
    if task == TASK_BEDBATH:            # BedBathingPR2: the wipe-target bit set and the target count
        L.update(T_WIPE=17, T_NTGT=23, MAX_TARGETS=160)
    return _Layout(**L)


SI = _scratch_layout()
BB = _scratch_layout(TASK_BEDBATH)


# DressingJaco-v0 (build-defined, include/avr_dressing.h): its constants and state layout, from
# the module avr.build generates from the header (so the package needs no header at import time)
from ._dressing_consts import DEFINES as _DRH  # noqa: E402
DR = _Layout(TASK=TASK_DRESSING, ACT_DIM=7, INFO_DIM=2, **{k[len('AVR_DR_'):]: v for k, v in _DRH.items()})
DR.STATE_WORDS = _DRH['AVR_DR_STATE_WORDS']
DR.OBS_DIM = _DRH['AVR_DR_OBS_DIM']
DR.S_TASK, DR.T_ITER, DR.T_FLAGS, DR.T_SUCCESS = _DRH['AVR_DR_S_TASK'], _DRH['AVR_DR_T_ITER'], _DRH['AVR_DR_T_FLAGS'], _DRH['AVR_DR_T_SUCCESS']
LAYOUTS = {TASK_FEEDING: FEEDING, TASK_SCRATCH: SI, TASK_BEDBATH: BB, TASK_DRESSING: DR}

PI32 = C.POINTER(C.c_int32)
PF64 = C.POINTER(C.c_double)


class avr_model_desc(C.Structure):
    _fields_ = [
        ('n_links', C.c_int32), ('n_dof', C.c_int32),
        ('rl_parent', PI32), ('rl_jtype', PI32), ('rl_dof', PI32), ('rl_has_limit', PI32),
        ('rl_jpos', PF64), ('rl_jquat', PF64), ('rl_axis', PF64),
        ('rl_com_pos', PF64), ('rl_com_quat', PF64), ('rl_mass', PF64), ('rl_inertia', PF64),
        ('rl_lower', PF64), ('rl_upper', PF64),
        ('robot_base', PF64),
        ('n_free', C.c_int32),
        ('fb_mass', PF64), ('fb_inertia', PF64), ('fb_gravity', PF64),
        ('n_static', C.c_int32),
        ('st_pose', PF64),
        ('n_human', C.c_int32),
        ('n_bodies', C.c_int32),
        ('body_kind', PI32), ('body_index', PI32), ('body_shape_start', PI32), ('body_shape_count', PI32),
        ('body_flags', PI32),
        ('body_friction', PF64), ('body_threshold', PF64),
        ('body_aabb', PF64),
        ('n_shapes', C.c_int32),
        ('shape_kind', PI32), ('shape_body', PI32), ('shape_gender', PI32), ('shape_hull', PI32),
        ('shape_pose', PF64), ('shape_param', PF64), ('shape_margin', PF64), ('shape_aabb', PF64),
        ('n_hull_verts', C.c_int32), ('n_hull_planes', C.c_int32),
        ('hull_verts', PF64), ('hull_planes', PF64),
        ('n_pairs', C.c_int32),
        ('pair_a', PI32), ('pair_b', PI32),
        ('n_arm', C.c_int32), ('arm_dofs', C.c_int32 * 8),
        ('n_finger', C.c_int32), ('finger_dofs', C.c_int32 * 4),
        ('tool_link', C.c_int32), ('torso_link', C.c_int32), ('head_slot', C.c_int32),
        ('spoon_free', C.c_int32), ('bowl_free', C.c_int32), ('food_free0', C.c_int32), ('n_food', C.c_int32),
        ('table_body', C.c_int32), ('bowl_body', C.c_int32), ('spoon_body', C.c_int32), ('food_body0', C.c_int32),
        ('human_body0', C.c_int32), ('n_human_bodies', C.c_int32), ('robot_body0', C.c_int32), ('n_robot_bodies', C.c_int32),
        ('tool_offset', C.c_double * 7),
        ('mouth_offset', (C.c_double * 3) * 2),
        ('arm_lower', C.c_double * 8), ('arm_upper', C.c_double * 8),
        ('time_step', C.c_double),
        ('num_sub_steps', C.c_int32), ('frame_skip', C.c_int32), ('solver_iterations', C.c_int32),
        ('max_episode_steps', C.c_int32),
        ('erp', C.c_double), ('warmstart', C.c_double), ('linear_damping', C.c_double),
        ('angular_damping', C.c_double), ('max_coord_vel', C.c_double),
        ('default_motor_impulse', C.c_double),
        ('robot_gain', C.c_double), ('robot_force', C.c_double),
        ('finger_gain', C.c_double), ('finger_force', C.c_double), ('finger_target', C.c_double),
        ('fixed_max_force', C.c_double),
        ('w_distance', C.c_double), ('w_action', C.c_double), ('w_food', C.c_double),
        ('w_velocity', C.c_double), ('w_force_nontarget', C.c_double), ('w_high_forces', C.c_double),
        ('w_food_hit', C.c_double), ('w_food_velocities', C.c_double), ('task_success_threshold', C.c_double),
        ('hc_n', C.c_int32), ('hc_parent_slot', C.c_int32),
        ('hc_slot', C.c_int32 * DESC_HC), ('hc_body', C.c_int32 * DESC_HC),
        ('hc_jpos', ((C.c_double * 3) * DESC_HC) * 2),
        ('hc_axis', (C.c_double * 3) * DESC_HC),
        ('hc_mass', (C.c_double * DESC_HC) * 2), ('hc_inertia', ((C.c_double * 3) * DESC_HC) * 2),
        ('hc_lower', C.c_double * DESC_HC), ('hc_upper', C.c_double * DESC_HC),
        ('human_gain', C.c_double), ('human_force', C.c_double),
        ('n_pairs_base', C.c_int32),
        # ABI 3
        ('task', C.c_int32), ('n_rstatic', C.c_int32),
        ('human_gravity', C.c_double * 3), ('fix_pivot_b', C.c_double * 3), ('tool_tip', C.c_double * 3),
        ('torso_com', C.c_double * 3), ('tool_handle_shapes', C.c_int32),
        ('w_tool_force', C.c_double), ('w_scratch', C.c_double),
        ('robot_gravity', C.c_double * 3),
        # ABI 4
        ('bb_targets', PF64), ('bb_ntgt', (C.c_int32 * 2) * 2), ('bb_limb_slots', C.c_int32 * 2),
        ('bb_joint_slots', C.c_int32 * 3), ('w_wipe', C.c_double), ('closest_distance', C.c_double),
        ('body_rolling', PF64), ('body_spinning', PF64),
    ]


# FeedingJaco physics / task constants.  Values marked [ext] are assumed Bullet/PyBullet
# defaults; the rest are cited to the reference.
FEEDING_PARAMS = dict(
    time_step=0.02,              # world_creation.py:75
    num_sub_steps=2,             # feeding.py:289
    frame_skip=5,                # feeding.py:18
    solver_iterations=10,        # feeding.py:289
    max_episode_steps=200,       # assistive_gym/__init__.py:270-274
    erp=0.2,                     # [ext] btContactSolverInfo::m_erp
    warmstart=0.85,              # [ext] btContactSolverInfo::m_warmstartingFactor
    linear_damping=0.04,         # [ext] btMultiBody default damping
    angular_damping=0.04,        # [ext]
    max_coord_vel=100.0,         # [ext] btMultiBody::m_maxCoordinateVelocity
    default_motor_impulse=1.0,   # [ext] PyBullet createJointMotors default velocity motor
    robot_gain=0.005,            # config.ini:21 (feeding robot_gains)
    robot_force=1.0,             # config.ini:22
    finger_gain=0.05,            # world_creation.py:328
    finger_force=500.0,          # world_creation.py:328
    finger_target=1.33,          # feeding.py:279
    fixed_max_force=500.0,       # world_creation.py:364
    w_distance=1.0, w_action=0.01, w_food=1.0,                       # config.ini:23-25
    w_velocity=0.25, w_force_nontarget=0.01, w_high_forces=0.05,     # config.ini:37-39
    w_food_hit=1.0, w_food_velocities=1.0,                           # config.ini:40-41
    task_success_threshold=0.75,                                     # config.ini:26
    human_gain=0.005,            # feeding.py:48 take_step(..., human_gains=0.005)
    human_force=1.0,             # feeding.py:17 human_forces (x human_strength, 1.0 unless 'weakness')
)


# ScratchItchPR2 physics / task constants ([ext]: assumed Bullet/PyBullet defaults, as above)
SCRATCH_PARAMS = dict(
    time_step=0.02,              # world_creation.py:75
    num_sub_steps=0,             # scratch_itch.py:258 (0: one step of time_step)
    frame_skip=5,                # scratch_itch.py:18
    solver_iterations=50,        # scratch_itch.py:258
    max_episode_steps=200,       # assistive_gym/__init__.py (ScratchItchPR2-v0)
    erp=0.2, warmstart=0.85, linear_damping=0.04, angular_damping=0.04, max_coord_vel=100.0,   # [ext]
    default_motor_impulse=1.0,   # [ext]
    robot_gain=0.05,             # config.ini:5 (scratch_itch robot_gains)
    robot_force=1.0,             # config.ini:4
    finger_gain=0.05,            # world_creation.py:328
    finger_force=500.0,          # world_creation.py:328
    finger_target=0.25,          # scratch_itch.py:192 set_gripper_open_position(position=0.25)
    fixed_max_force=500.0,       # world_creation.py:364
    w_distance=1.0, w_action=0.01, w_food=0.0,                       # config.ini:6-7
    w_tool_force=0.01, w_scratch=2.0,                                # config.ini:8-9
    w_velocity=0.25, w_force_nontarget=0.01, w_high_forces=0.05,     # config.ini:37-39
    w_food_hit=0.0, w_food_velocities=0.0,
    task_success_threshold=25.0,                                     # config.ini:10
    human_gain=0.05,             # scratch_itch.py:45 take_step(..., human_gains=0.05) under 'tremor'
    human_force=1.0,             # env.py:274 take_step default human_forces (x human_strength)
    reactive_gain=0.01,          # scratch_itch.py:263 human_reactive_gain (not a descriptor field)
    reactive_force=1.0,          # scratch_itch.py:263 human_reactive_force (x human_strength)
)

# BedBathingPR2 physics / task constants
BEDBATH_PARAMS = dict(SCRATCH_PARAMS)
BEDBATH_PARAMS.update(
    solver_iterations=50,        # bed_bathing.py:338 (numSubSteps=0, numSolverIterations=50)
    robot_gain=0.05,             # config.ini:14 (bed_bathing robot_gains)
    robot_force=1.0,             # config.ini:13
    finger_target=0.2,           # bed_bathing.py:319 set_gripper_open_position(position=0.2)
    w_distance=1.0, w_action=0.01,                                   # config.ini:15-16
    w_tool_force=0.0, w_scratch=0.0,
    w_wipe=5.0,                  # config.ini:17 wiping_reward_weight
    task_success_threshold=0.3,  # config.ini:18 (x total_target_count, bed_bathing.py:70)
    human_gain=0.05,             # bed_bathing.py:46 take_step(..., human_gains=0.05) (no tremor: impairment 'none')
    closest_distance=4.0,        # bed_bathing.py:61 getClosestPoints(..., distance=4.0)
    settle_motor_force=0.1,      # world_creation.py:164-166: bed_bathing human joints VELOCITY_CONTROL force 0.1 (reset settle)
    settle_frames=100,           # bed_bathing.py:288-289
)
HOST_ONLY_PARAMS = ('reactive_gain', 'reactive_force', 'settle_motor_force', 'settle_frames')

SCENES = {TASK_FEEDING: 'feeding_jaco', TASK_SCRATCH: 'scratch_itch_pr2', TASK_BEDBATH: 'bed_bathing_pr2'}


def load_scene(name='feeding_jaco'):
    if isinstance(name, int):
        name = SCENES[name]
    return dict(np.load(os.path.join(DATA_DIR, name + '.npz')))


def scene_task(A):
    if 'task_dressing' in A:
        return TASK_DRESSING
    if 'bb_targets' in A:
        return TASK_BEDBATH
    return TASK_SCRATCH if 'n_rstatic' in A else TASK_FEEDING


class ModelDesc:
    """Owns the arrays behind an `avr_model_desc`."""

    def __init__(self, A, params=None):
        task = scene_task(A)
        P = dict({TASK_SCRATCH: SCRATCH_PARAMS, TASK_BEDBATH: BEDBATH_PARAMS}.get(task, FEEDING_PARAMS))
        if params:
            P.update(params)
        self.task = task
        self.layout = LAYOUTS[task]
        self.A = {}
        self.params = P
        d = avr_model_desc()

        def arr(key, dtype):
            a = np.ascontiguousarray(A[key], dtype=dtype)
            if a.size == 0:
                a = np.zeros(1, dtype=dtype)
            self.A[key] = a
            return a.ctypes.data_as(PI32 if dtype == np.int32 else PF64)

        d.n_links = int(A['n_links'])
        d.n_dof = int(A['n_dof'])
        for k in ('rl_parent', 'rl_jtype', 'rl_dof', 'rl_has_limit'):
            setattr(d, k, arr(k, np.int32))
        for k in ('rl_jpos', 'rl_jquat', 'rl_axis', 'rl_com_pos', 'rl_com_quat', 'rl_mass', 'rl_inertia',
                  'rl_lower', 'rl_upper', 'robot_base'):
            setattr(d, k, arr(k, np.float64))
        d.n_free = len(A['fb_mass'])
        for k in ('fb_mass', 'fb_inertia', 'fb_gravity'):
            setattr(d, k, arr(k, np.float64))
        d.n_static = len(A['st_pose'])
        d.st_pose = arr('st_pose', np.float64)
        d.n_human = len(A['human_slot_link'])
        d.n_bodies = len(A['body_kind'])
        for k in ('body_kind', 'body_index', 'body_shape_start', 'body_shape_count', 'body_flags'):
            setattr(d, k, arr(k, np.int32))
        for k in ('body_friction', 'body_threshold', 'body_aabb'):
            setattr(d, k, arr(k, np.float64))
        for k in ('body_rolling', 'body_spinning'):          # (scenes compiled before ABI 5: none)
            if k in A:
                setattr(d, k, arr(k, np.float64))
            else:
                self.A[k] = np.zeros(d.n_bodies)
                setattr(d, k, self.A[k].ctypes.data_as(PF64))
        d.n_shapes = len(A['shape_kind'])
        for k in ('shape_kind', 'shape_body', 'shape_gender', 'shape_hull'):
            setattr(d, k, arr(k, np.int32))
        for k in ('shape_pose', 'shape_param', 'shape_margin', 'shape_aabb'):
            setattr(d, k, arr(k, np.float64))
        d.n_hull_verts = len(A['hull_verts'])
        d.n_hull_planes = 0
        d.hull_verts = arr('hull_verts', np.float64)
        self.A['hull_planes'] = np.zeros(4)
        d.hull_planes = self.A['hull_planes'].ctypes.data_as(PF64)
        d.n_pairs = len(A['pair_a'])
        d.n_pairs_base = int(A['n_pairs_base']) if 'n_pairs_base' in A else d.n_pairs
        d.pair_a = arr('pair_a', np.int32)
        d.pair_b = arr('pair_b', np.int32)
        arm = [int(x) for x in A['task_arm_dofs']]
        fin = [int(x) for x in A['task_finger_dofs']]
        d.n_arm = len(arm)
        for i, x in enumerate(arm):
            d.arm_dofs[i] = x
        d.n_finger = len(fin)
        for i, x in enumerate(fin):
            d.finger_dofs[i] = x
        d.tool_link = int(A['task_tool_link'])
        if task == TASK_FEEDING:
            d.torso_link = int(A['task_torso_link'])
            d.head_slot = int(A['task_head_slot'])
        d.task = task
        if task in (TASK_SCRATCH, TASK_BEDBATH):
            d.spoon_free, d.bowl_free, d.food_free0, d.n_food = 0, -1, -1, 0
            d.table_body = d.bowl_body = d.food_body0 = -1
            d.spoon_body = int(A['task_tool_body'])
            d.n_rstatic = int(A['n_rstatic'])
            d.human_gravity[2] = -1.0                    # scratch_itch.py:260; bed_bathing.py:286 (the reset settle)
            for i in range(3):
                d.fix_pivot_b[i] = float(A['task_tool_pivot'][i])
                d.tool_tip[i] = float(A['task_tool_tip'][i])
                d.torso_com[i] = float(A['task_torso_com'][i])
            d.tool_handle_shapes = int(A['task_tool_handle_shapes'])
            d.torso_link = -1
            d.head_slot = -1
            if task == TASK_BEDBATH:
                d.bb_targets = arr('bb_targets', np.float64)
                for g in range(2):
                    for l in range(2):
                        d.bb_ntgt[g][l] = int(A['bb_ntgt'][g][l])
                for i in range(2):
                    d.bb_limb_slots[i] = int(A['bb_limb_slots'][i])
                for i in range(3):
                    d.bb_joint_slots[i] = int(A['bb_joint_slots'][i])
        else:
            d.spoon_free, d.bowl_free, d.food_free0, d.n_food = 0, 1, 2, 8
            d.table_body = int(A['task_table_body'])
            d.bowl_body = int(A['task_bowl_body'])
            d.spoon_body = int(A['task_spoon_body'])
            d.food_body0 = int(A['task_food_body0'])
        d.human_body0 = int(A['task_human_body0'])
        d.n_human_bodies = int(np.sum(A['body_kind'] == 3))
        d.robot_body0 = 0
        d.n_robot_bodies = int(np.sum(A['body_kind'] == 0))
        for i, x in enumerate(A['task_tool_offset']):
            d.tool_offset[i] = float(x)
        if task == TASK_FEEDING:
            for i in range(3):
                d.mouth_offset[0][i] = float(A['task_mouth_male'][i])
                d.mouth_offset[1][i] = float(A['task_mouth_female'][i])
        # take_step limit zeroing uses getJointInfo limits; continuous joints -> +-1e10
        # (world_creation.py:122-124)
        dof_link = {int(A['rl_dof'][l]): l for l in range(int(A['n_links'])) if A['rl_dof'][l] >= 0}
        for i, dof in enumerate(arm):
            l = dof_link[dof]
            if A['rl_has_limit'][l]:
                d.arm_lower[i], d.arm_upper[i] = float(A['rl_lower'][l]), float(A['rl_upper'][l])
            else:
                d.arm_lower[i], d.arm_upper[i] = -1e10, 1e10
        if 'hc_slot' in A:                 # articulated human chain (model_compiler.head_chain)
            nhc = int(A['hc_n']) if 'hc_n' in A else HC_N
            d.hc_n = nhc
            d.hc_parent_slot = int(A['hc_parent_slot'])
            for k in range(nhc):
                d.hc_slot[k] = int(A['hc_slot'][k])
                d.hc_body[k] = int(A['hc_body'][k])
                d.hc_lower[k] = float(A['hc_lower'][k])
                d.hc_upper[k] = float(A['hc_upper'][k])
                for i in range(3):
                    d.hc_axis[k][i] = float(A['hc_axis'][k][i])
                for g in range(2):
                    d.hc_mass[g][k] = float(A['hc_mass'][g][k])
                    for i in range(3):
                        d.hc_jpos[g][k][i] = float(A['hc_jpos'][g][k][i])
                        d.hc_inertia[g][k][i] = float(A['hc_inertia'][g][k][i])
        for k, v in P.items():
            if k in HOST_ONLY_PARAMS:
                continue
            if k == 'robot_gravity':
                for i in range(3):
                    d.robot_gravity[i] = float(v[i])
                continue
            setattr(d, k, v)
        self.desc = d
        self.n_dof = d.n_dof
        self.arm_dofs = arm
        self.finger_dofs = fin
        self.dof_link = dof_link

    def ptr(self):
        return C.byref(self.desc)
