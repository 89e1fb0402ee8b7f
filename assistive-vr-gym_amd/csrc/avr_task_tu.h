// avr_task_tu.h -- one task's instantiation of the step kernels (avr_kernel.hip) and the C-ABI
// body (avr_capi.hip) inside namespace AVR_NS.  Everything with external linkage (kernels, launch
// helpers, the per-task API functions) lives in that namespace, so the FeedingJaco and ScratchItch
// instantiations link into one libavr.so side by side; avr_api.cpp exports the C entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/avr.h"

namespace AVR_NS {
#include "avr_math.h"
#include "avr_kmodel.h"
#include "avr_kernel.hip"
#include "avr_reset_ik.hip"
#include "avr_base_search.hip"
#include "avr_capi.hip"
}  // namespace AVR_NS
