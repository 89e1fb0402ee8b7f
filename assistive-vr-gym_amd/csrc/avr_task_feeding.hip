// FeedingJaco-v0 instantiation of the step kernels and the C-ABI body (avr_task_tu.h).
#define AVR_TASK AVR_TASK_FEEDING
#define AVR_NS avr_feeding
#include "avr_task_tu.h"
