// Internal hooks of the native Prophet scheduler (HIP-free) for the PUSH loop
// (bpsr_prophet_loop.cpp).
#pragma once

#include <cstddef>
#include <vector>

#include "bpsr/prophet.h"

namespace bpsr {
// One getTask() poll under the queue's lock: 1 and *out when a task is
// released, else 0; *progressed tells whether the poll changed any state.
int prophet_poll(byteps_prophet_queue* q, byteps_prophet_task* out, bool* progressed);
// Add n tasks under one lock (all or nothing: a bad task adds none).
int prophet_add_many(byteps_prophet_queue* q, const byteps_prophet_task* t, size_t n);
// Poll under one lock until a poll makes no progress, appending the released
// tasks to *released; at each release group's end the group's partitions are
// reported finished (credit back, as byteps_prophet_report_finish).  Returns
// the number released.
size_t prophet_drain(byteps_prophet_queue* q, std::vector<byteps_prophet_task>* released);
}  // namespace bpsr
