// Internal hooks of the native Prophet scheduler (HIP-free) for the PUSH loop
// (bpsr_prophet_loop.cpp).
#pragma once

#include "bpsr/prophet.h"

namespace bpsr {
// One getTask() poll under the queue's lock: 1 and *out when a task is
// released, else 0; *progressed tells whether the poll changed any state.
int prophet_poll(byteps_prophet_queue* q, byteps_prophet_task* out, bool* progressed);
}  // namespace bpsr
