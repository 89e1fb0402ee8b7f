/* avr_dressing.h -- DressingJaco-v0 (BASELINE configs[4]): constants and the per-env state layout
 * shared by the gfx950 kernel (assistive-vr-gym_amd/csrc/avr_dressing.hip) and the CPU oracle
 * (oracle/avr_oracle_dressing.c).
 *
 * A BUILD-DEFINED task.  The reference has no dressing environment; it holds only the
 * hooks this task is built on:
 *   - the cloth collision spheres at the shoulder, elbow and wrist (human_creation.py:90-95 male,
 *     136-141 female; links 18, 20, 22 of the left arm, human_creation.py:214-219);
 *   - the dressing-force preference term reward_dressing_force = -sum |dressing_forces|
 *     (env.py:433-434, weight dressing_force_weight 0.01, config.ini:43);
 *   - Util.sleeve_on_arm_reward (util.py:188-252) and line_intersects_triangle (util.py:179-186).
 * Everything else -- the sleeve's mass-spring model, its penalty contact against the arm, the
 * kinematically driven Jaco, the reward's task terms and the observation -- is this build's
 * definition, documented in DESIGN.md section 10; there is no parity anchor beyond the oracle.
 *
 * Per env step (take_step, env.py:274-351 semantics for the 7 Jaco arm joints): frame_skip 5 frames
 * of 0.02 s; per frame 2 robot sub-steps of 0.01 s (the arm joints follow their POSITION_CONTROL
 * targets by the unsaturated motor's closed form q += kp (q* - q), test_motor_row_closed_form), each
 * with AVR_DR_CSUB cloth sub-steps of 1 ms (the held cuff ring moves with the tool frame,
 * interpolated across the robot sub-step; free particles: springs, gravity, damping, penalty
 * contact with the arm, semi-implicit Euler).
 */
#ifndef AVR_DRESSING_H
#define AVR_DRESSING_H

#define AVR_DR_RINGS 8                 /* sleeve rings along its axis (ring 0 = the held cuff)      */
#define AVR_DR_SEGS 16                 /* particles around a ring                                    */
#define AVR_DR_NP (AVR_DR_RINGS * AVR_DR_SEGS)   /* 128 particles                                    */
#define AVR_DR_RADIUS 0.07             /* sleeve radius (m): the male hand sphere 0.043 passes       */
#define AVR_DR_SPACING 0.035           /* ring spacing (m): a 0.245 m sleeve                         */
#define AVR_DR_MASS 0.1                /* sleeve mass (kg), spread evenly over the particles         */
#define AVR_DR_K_STRUCT 100.0          /* spring stiffness (N/m): ring and axial neighbours           */
#define AVR_DR_K_SHEAR 50.0            /*   diagonal neighbours                                       */
#define AVR_DR_K_BEND 5.0              /*   second neighbours along the ring and the axis             */
#define AVR_DR_DAMP 0.05               /* spring damping (N s/m) along each spring                    */
#define AVR_DR_AIR 0.02                /* air drag (N s/m) per particle                               */
#define AVR_DR_GRAVITY (-9.81)
#define AVR_DR_K_CONTACT 200.0         /* penalty contact stiffness (N/m)                             */
#define AVR_DR_C_CONTACT 0.2           /* penalty contact damping (N s/m), approaching only           */
#define AVR_DR_THICK 0.005             /* cloth thickness (m): contact at shape radius + thickness    */
#define AVR_DR_CSUB 10                 /* cloth sub-steps per robot sub-step                          */
#define AVR_DR_RSUB 2                  /* robot sub-steps per frame (numSubSteps 2, as FeedingJaco)   */
#define AVR_DR_FRAME 0.02              /* s per frame (world_creation.py:75)                          */
#define AVR_DR_FRAME_SKIP 5
#define AVR_DR_MAX_STEPS 200           /* TimeLimit                                                   */
#define AVR_DR_ARM 7                   /* Jaco arm joints 1..7 (world_creation.py:283)                */
#define AVR_DR_KP 0.05                 /* arm motor gain (scratch_itch / bed_bathing robot_gains)     */
#define AVR_DR_NSHAPE 6                /* contact shapes: upper-arm capsule, forearm capsule, hand
                                          sphere, shoulder / elbow / wrist cloth spheres              */
/* reward weights: action_weight 0.01 (config.ini), velocity 0.25 (config.ini:37),
 * dressing_force_weight 0.01 (config.ini:43); distance and dressing progress 1.0 (build-defined) */
#define AVR_DR_W_DISTANCE 1.0
#define AVR_DR_W_ACTION 0.01
#define AVR_DR_W_DRESS 1.0
#define AVR_DR_W_VELOCITY 0.25
#define AVR_DR_W_FORCE 0.01
#define AVR_DR_OBS_DIM 24

/* ---- per-env state block (floats) ---- */
#define AVR_DR_S_Q 0                   /* [7] arm joint positions (Jaco DoFs 0..6)                    */
#define AVR_DR_S_QT 8                  /* [7] arm motor targets                                       */
#define AVR_DR_S_GEO 16                /* [32] arm geometry (world, static per episode):
                                          +0 shoulder, +3 elbow, +6 wrist, +9 hand centre (points),
                                          +12 upper-arm capsule a, +15 b, +18 its radius,
                                          +19 forearm capsule a, +22 b, +25 radius, +26 hand radius,
                                          +27 shoulder / +28 elbow / +29 wrist cloth-sphere radii     */
#define AVR_DR_S_TASK 48               /* [16] task words                                            */
#define AVR_DR_T_ITER 0                /*   env steps this episode                                   */
#define AVR_DR_T_GENDER 1              /*   0 male, 1 female                                         */
#define AVR_DR_T_SUCCESS 2             /*   upper arm in the sleeve (last step)                      */
#define AVR_DR_T_FLAGS 3               /*   bit 0: non-finite state                                  */
#define AVR_DR_T_FORCE 4               /*   sum |dressing force| of the last cloth sub-step (N)      */
#define AVR_DR_T_FOREARM 5             /*   forearm in the sleeve (last step)                        */
#define AVR_DR_S_TOOL 64               /* [8] tool (end-effector COM) frame: pos 3, quat 4           */
#define AVR_DR_S_X 80                  /* [NP][4] particle positions (w unused)                      */
#define AVR_DR_S_V (AVR_DR_S_X + 4 * AVR_DR_NP)   /* [NP][4] particle velocities                     */
#define AVR_DR_STATE_WORDS (AVR_DR_S_V + 4 * AVR_DR_NP)   /* 1104 */

#endif
