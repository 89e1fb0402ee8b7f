// avr_task.h -- compile-time task configuration of one instantiation of the step kernels and the
// C-ABI body (avr_task_feeding.hip / avr_task_scratch.hip include the shared sources once each,
// inside their own namespace).  AVR_TASK selects the state layout of include/avr_model.h and the
// task glue; the shared sources use only the K_ / S_ / T_ names defined here.
#pragma once
#include "../../include/avr_model.h"

#ifndef AVR_TASK
#error "AVR_TASK must be defined (AVR_TASK_FEEDING, AVR_TASK_SCRATCH or AVR_TASK_BEDBATH)"
#endif

#define T_TARGET 0      // task words common to both layouts
#define T_ITER 3
#define T_SUCCESS 4
#define T_GENDER 7
#define T_FLAGS 8
#define T_NCP 9
#define T_HDYN 10
#define T_COOPN 15      // consecutive sub-steps with more than AVR_COOP_CAP EPAs (avr_kernel.hip np_coop)

#if AVR_TASK == AVR_TASK_FEEDING
#define K_MAX_LINKS AVR_MAX_LINKS
#define K_MAX_DOF AVR_MAX_DOF
#define K_HC_N AVR_HC_N
#define K_MAX_FREE AVR_MAX_FREE
#define K_MAX_HUMAN AVR_MAX_HUMAN
#define K_MAX_CONTACTS AVR_MAX_CONTACTS
#define K_ACT_DIM AVR_ACT_DIM
#define K_OBS_DIM AVR_OBS_DIM
#define S_Q AVR_S_Q
#define S_QD AVR_S_QD
#define S_QTGT AVR_S_QTGT
#define S_KP AVR_S_KP
#define S_MAXIMP AVR_S_MAXIMP
#define S_FREE AVR_S_FREE
#define S_TASK AVR_S_TASK
#define S_HUMAN AVR_S_HUMAN
#define S_HCH AVR_S_HCH
#define S_CP AVR_S_CP
#define K_STATE_WORDS AVR_STATE_WORDS
#define K_T_WORDS AVR_T_WORDS
#define T_ALIVE AVR_T_ALIVE
#define T_HIT AVR_T_HIT
#define K_RBASE_IN_STATE 0      // robot base: a model constant (feeding.py:188)
#define K_CHAIN_LIMITS_IN_STATE 0
#define K_HUMAN_GRAVITY 0       // robot, human and spoon gravity are 0 (feeding.py:285-287)
#define K_TOOL_PIVOT 0          // the spoon's base COM is its body frame
#define K_PR2 0
#define K_ND 10                 // robot DoFs (Jaco); the articulated human chain's DoFs follow
#define K_TORSION 0             // no rolling / spinning friction in the FeedingJaco scene
#elif AVR_TASK == AVR_TASK_SCRATCH || AVR_TASK == AVR_TASK_BEDBATH
// the PR2 family: ScratchItchPR2 and BedBathingPR2 share the state layout (AVR_SI_*)
#define K_PR2 1
#define K_ND 14                 // robot DoFs (PR2 left-arm subtree); the human arm chain's DoFs follow
#define K_MAX_LINKS AVR_SI_MAX_LINKS
#define K_MAX_DOF AVR_SI_MAX_DOF
#define K_HC_N AVR_SI_HC_N
#define K_MAX_FREE AVR_SI_MAX_FREE
#define K_MAX_HUMAN AVR_SI_MAX_HUMAN
#define K_MAX_CONTACTS AVR_SI_MAX_CONTACTS
#define K_ACT_DIM AVR_SI_ACT_DIM
#if AVR_TASK == AVR_TASK_BEDBATH
#define K_OBS_DIM AVR_BB_OBS_DIM
#define T_WIPE AVR_BB_T_WIPE
#define T_NTGT AVR_BB_T_NTGT
#else
#define K_OBS_DIM AVR_SI_OBS_DIM
#endif
#define S_Q AVR_SI_S_Q
#define S_QD AVR_SI_S_QD
#define S_QTGT AVR_SI_S_QTGT
#define S_KP AVR_SI_S_KP
#define S_MAXIMP AVR_SI_S_MAXIMP
#define S_FREE AVR_SI_S_FREE
#define S_RBASE AVR_SI_S_RBASE
#define S_TASK AVR_SI_S_TASK
#define S_HUMAN AVR_SI_S_HUMAN
#define S_HCH AVR_SI_S_HCH
#define S_CP AVR_SI_S_CP
#define K_STATE_WORDS AVR_SI_STATE_WORDS
#define K_T_WORDS AVR_SI_T_WORDS
#define T_LIMB AVR_SI_T_LIMB
#define T_STRENGTH AVR_SI_T_STRENGTH
#define T_PREV AVR_SI_T_PREV
#define T_TREMOR AVR_SI_T_TREMOR
#define T_ONARM AVR_SI_T_ONARM
#define K_RBASE_IN_STATE 1      // PR2 base pose per env (position_robot_toc, env.py:489-585)
#define K_CHAIN_LIMITS_IN_STATE 1   // human arm limits x limit_scale per env (human_creation.py:226)
#define K_HUMAN_GRAVITY 1       // human gravity -1 (scratch_itch.py:260; BedBathing's reset settle, bed_bathing.py:286)
#define K_TOOL_PIVOT 1          // the scratcher / wiper is a composite body: its handle COM is off the body frame
#define K_TORSION 1             // torsional friction rows: the tools' rolling / spinning friction 0.001
                                // (tool_scratch.urdf:22-25, wiper.urdf:21-24), the bed parts' 5 / 5
                                // (bed_bathing.py:282)
#else
#error "unknown AVR_TASK"
#endif
// constraint rows per contact point: the normal and two lateral frictions, then (K_TORSION) the
// spinning row about the normal and two rolling rows about the friction directions
#define K_CROWS (K_TORSION ? 6 : 3)
