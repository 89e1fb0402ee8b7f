// BedBathingPR2-v0 instantiation of the step kernels and the C-ABI body (avr_task_tu.h).
#define AVR_TASK AVR_TASK_BEDBATH
#define AVR_NS avr_bedbath
#include "avr_task_tu.h"
