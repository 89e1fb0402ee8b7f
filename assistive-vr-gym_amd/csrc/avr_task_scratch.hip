// ScratchItchPR2-v0 instantiation of the step kernels and the C-ABI body (avr_task_tu.h).
#define AVR_TASK AVR_TASK_SCRATCH
#define AVR_NS avr_scratch
#include "avr_task_tu.h"
