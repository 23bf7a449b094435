// Prophet's PUSH-stage scheduler, native (include/bpsr/prophet.h).
//
// State follows BytePSScheduledQueue for the PUSH queue
// (byteps/common/scheduled_queue.cc:217-296, scheduled_queue.h:77-95) with
// containers that fit the access pattern: the priority multiset becomes one
// FIFO of queued partitions per gradient (findTask is always an exact-priority
// lookup, and equal priorities keep insertion order) — a vector and a head
// index that keep their capacity, so a steady-state iteration allocates
// nothing — the 160-entry arrays are sized by the model's last checkpoint, the
// stack holds gradient indices.
#include <climits>
#include <cmath>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <vector>

#include "bpsr/prophet.h"
#include "bpsr_error.h"
#include "bpsr_prophet_internal.h"

namespace {

// scheduled_queue.h:81-85
constexpr int32_t kRefCheckpoints[13] = {-1, 9, 22, 35, 50, 62, 77, 90, 103, 117, 130, 143, 156};
constexpr double kRefExec[13] = {16, 15, 9, 10, 12, 18, 15, 21, 30, 25, 20, 5, 0};

}  // namespace

struct byteps_prophet_queue {
  std::mutex mu;
  std::vector<int32_t> checkpoints;
  std::vector<double> budget;           // per block, bytes (constructor, :26-33)
  int64_t credit0 = 0;
  // queued tasks: per gradient (_ms) a FIFO = vector + head (emptied -> cleared)
  struct Fifo {
    std::vector<byteps_prophet_task> v;
    size_t head = 0;
    bool empty() const { return head == v.size(); }
    const byteps_prophet_task& front() const { return v[head]; }
    void push_back(const byteps_prophet_task& t) { v.push_back(t); }
    void pop_front() {
      if (++head == v.size()) {
        v.clear();
        head = 0;
      }
    }
  };
  std::vector<Fifo> tasks;
  std::vector<int32_t> tensor_part;                    // _tensor_part
  std::deque<byteps_prophet_task> fifo;                // _sq
  uint64_t nsched = 0;                                 // _ms.size()
  // iteration state
  int32_t pointer = 0, expected = 0, sizepointer = 0;
  bool dequeue = false, meetzero = false;
  double dynamic = 0;
  int64_t credit = 0;
  std::vector<char> visited;
  std::vector<int32_t> stack;
  int32_t phase = BYTEPS_PROPHET_CREDIT;

  void reset() {
    pointer = (int32_t)checkpoints.size() - 1;
    expected = checkpoints[pointer];
    stack.clear();
    std::fill(visited.begin(), visited.end(), 0);
    dequeue = meetzero = false;
    sizepointer = 0;
    dynamic = 0;
    credit = credit0;
  }

  void end_block() {  // :245-251, :265-270
    dequeue = false;
    if (pointer > 0) --pointer;
  }

  const byteps_prophet_task* find(int32_t grad) const {
    if (grad < 0 || grad >= (int32_t)tasks.size() || tasks[grad].empty()) return nullptr;
    return &tasks[grad].front();
  }

  // one getTask() poll; returns true and fills *out when a task is released.
  // *progressed (if given): whether the poll changed any state — a poll that
  // returns no task may still advance collection or end a block, and the
  // next poll can then release without new input.
  bool poll(byteps_prophet_task* out, int32_t* ph, bool* progressed = nullptr) {
    bool dummy;
    bool& prog = progressed ? *progressed : dummy;
    prog = true;
    if (nsched == 0) {  // :292-318, the FIFO (no ready events / tables here)
      if (fifo.empty()) return prog = false;
      *out = fifo.front();
      fifo.pop_front();
      *ph = BYTEPS_PROPHET_FIFO;
      return true;
    }
    if (!dequeue) {  // collection, :221-241
      if (!find(expected)) return prog = false;
      if (!visited[expected]) {
        for (int32_t x = 0; x < tensor_part[expected]; ++x) {
          stack.push_back(expected);
          if (expected == 0) meetzero = true;
        }
        visited[expected] = 1;
      }
      if (expected >= 0) --expected;
      if (pointer > 0 && expected == checkpoints[pointer - 1]) {
        dequeue = true;
        dynamic = budget[sizepointer++];
      }
      return false;
    }
    if (stack.empty()) {  // the reference reads top() of the empty stack here
      end_block();
      return false;
    }
    const byteps_prophet_task* t = find(stack.back());
    if (!t) return prog = false;
    if (!meetzero) {  // budget, :261-271 (strict)
      if (dynamic > (double)t->len) {
        dynamic -= (double)t->len;
        phase = sizepointer - 1;
      } else {
        end_block();
        return false;
      }
    } else if (credit < t->len) {  // credit, :272-278
      return prog = false;
    } else {
      credit -= t->len;
      phase = BYTEPS_PROPHET_CREDIT;
    }
    *out = *t;
    tasks[stack.back()].pop_front();
    --nsched;
    stack.pop_back();
    *ph = phase;
    if (stack.empty() && meetzero) reset();  // :276-290 (phase survives)
    return true;
  }

  int validate(const byteps_prophet_task& t) const {
    if (t.len < 0) return bpsr::fail(BYTEPS_REDUCE_EARGS, "task length %lld < 0", (long long)t.len);
    if (!t.scheduled) return 0;
    if (t.grad < 0 || t.grad >= (int32_t)tasks.size())
      return bpsr::fail(BYTEPS_REDUCE_EARGS, "gradient %d outside [0, %d] (the last checkpoint)",
                        t.grad, (int)tasks.size() - 1);
    if (t.total_partnum < 1)
      return bpsr::fail(BYTEPS_REDUCE_EARGS, "total_partnum %d < 1", t.total_partnum);
    return 0;
  }

  int add(const byteps_prophet_task& t) {
    if (const int rc = validate(t)) return rc;
    if (!t.scheduled) {
      fifo.push_back(t);
      return 0;
    }
    tasks[t.grad].push_back(t);
    tensor_part[t.grad] = t.total_partnum;
    ++nsched;
    return 0;
  }
};

extern "C" {

int byteps_prophet_create(const byteps_prophet_config* cfg, byteps_prophet_queue** out) {
  if (!cfg || !out) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null config or output");
  *out = nullptr;
  std::vector<int32_t> cps;
  if (cfg->checkpoints) {
    if (cfg->ncheckpoints < 2) return bpsr::fail(BYTEPS_REDUCE_EARGS, "need >= 2 checkpoints");
    cps.assign(cfg->checkpoints, cfg->checkpoints + cfg->ncheckpoints);
  } else {
    cps.assign(kRefCheckpoints, kRefCheckpoints + 13);
  }
  if (cps[0] != -1) return bpsr::fail(BYTEPS_REDUCE_EARGS, "checkpoints[0] must be -1");
  for (size_t i = 1; i < cps.size(); ++i)
    if (cps[i] <= cps[i - 1]) return bpsr::fail(BYTEPS_REDUCE_EARGS, "checkpoints must ascend");
  if (!cfg->backward_exec && cps.size() != 13)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "custom checkpoints need their backward_exec");
  if (cfg->batch_size < 0 || cfg->net_b < 0 || cfg->credit < 0)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "batch_size, net_b and credit must be >= 0");
  auto* q = new (std::nothrow) byteps_prophet_queue;
  if (!q) return bpsr::fail(BYTEPS_REDUCE_EARGS, "out of memory");
  q->checkpoints = cps;
  // :27-33: B *= 125; exec *= (int)(batch / 64); exec *= B — same operation
  // order in double as prophet's restatement (oracle/prophet_oracle.py)
  const double scale = (double)(int64_t)((double)cfg->batch_size / 64);
  const double b = (double)(cfg->net_b * 125);
  for (size_t i = 0; i < cps.size(); ++i) {
    const double e = cfg->backward_exec ? cfg->backward_exec[i] : kRefExec[i];
    q->budget.push_back(e * scale * b);
  }
  q->credit0 = cfg->credit;
  const size_t ngrad = (size_t)cps.back() + 1;
  q->tasks.resize(ngrad);
  q->tensor_part.assign(ngrad, 0);
  q->visited.assign(ngrad, 0);
  q->reset();
  *out = q;
  return 0;
}

int byteps_prophet_destroy(byteps_prophet_queue* q) {
  delete q;
  return 0;
}

int byteps_prophet_add_task(byteps_prophet_queue* q, const byteps_prophet_task* t) {
  if (!q || !t) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null queue or task");
  std::lock_guard<std::mutex> g(q->mu);
  return q->add(*t);
}

int byteps_prophet_get_task(byteps_prophet_queue* q, byteps_prophet_task* out, int32_t* phase) {
  if (!q || !out) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null queue or output");
  std::lock_guard<std::mutex> g(q->mu);
  int32_t ph = 0;
  if (!q->poll(out, &ph)) return 0;
  if (phase) *phase = ph;
  return 1;
}

int byteps_prophet_report_finish(byteps_prophet_queue* q, int64_t size) {
  if (!q) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null queue");
  std::lock_guard<std::mutex> g(q->mu);
  if (size > 0 && q->meetzero) q->credit += size;  // :367-369
  return 0;
}

int byteps_prophet_pending(byteps_prophet_queue* q, uint64_t* n) {
  if (!q || !n) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null queue or output");
  std::lock_guard<std::mutex> g(q->mu);
  *n = q->nsched + q->fifo.size();
  return 0;
}

int byteps_prophet_get_state(byteps_prophet_queue* q, byteps_prophet_state* out) {
  if (!q || !out) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null queue or output");
  std::lock_guard<std::mutex> g(q->mu);
  out->pointer = q->pointer;
  out->expected = q->expected;
  out->sizepointer = q->sizepointer;
  out->dequeue = q->dequeue;
  out->meetzero = q->meetzero;
  out->stack_depth = (int32_t)q->stack.size();
  out->credit = q->credit;
  out->budget_left = q->dynamic;
  return 0;
}

int byteps_prophet_reset(byteps_prophet_queue* q) {
  if (!q) return bpsr::fail(BYTEPS_REDUCE_EARGS, "null queue");
  std::lock_guard<std::mutex> g(q->mu);
  q->reset();
  return 0;
}

int byteps_prophet_release_groups(byteps_prophet_queue* q, const byteps_prophet_task* arrivals,
                                  size_t n, int finish_immediately, int split_on_phase,
                                  uint64_t max_idle, byteps_prophet_task* released,
                                  int32_t* group_start, int32_t* group_phase) {
  if (!q || (n && (!arrivals || !released || !group_phase)) || !group_start)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "null queue or buffer");
  if (n > (size_t)INT32_MAX) return bpsr::fail(BYTEPS_REDUCE_EARGS, "too many arrivals");
  std::lock_guard<std::mutex> g(q->mu);
  // room for what is already queued as well: every release lands in released[]
  if (q->nsched + q->fifo.size() > 0)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "queue must be empty (%llu tasks pending)",
                      (unsigned long long)(q->nsched + q->fifo.size()));
  for (size_t i = 0; i < n; ++i)  // all or nothing: a bad arrival adds none
    if (const int rc = q->validate(arrivals[i])) return rc;
  size_t next = 0, nrel = 0;
  int32_t ngroups = 0, cur_phase = 0;
  bool open = false;  // a group is being filled
  uint64_t idle = 0;
  for (;;) {
    if (next < n) {
      const int rc = q->add(arrivals[next]);
      if (rc) return rc;
      ++next;
    }
    byteps_prophet_task t;
    int32_t ph = 0;
    if (q->poll(&t, &ph)) {
      if (open && split_on_phase && ph != cur_phase) {
        group_phase[ngroups++] = cur_phase;
        group_start[ngroups] = (int32_t)nrel;
        open = false;
      }
      if (!open) {
        group_start[ngroups] = (int32_t)nrel;
        open = true;
      }
      cur_phase = ph;
      released[nrel++] = t;
      idle = 0;
      if (finish_immediately && t.len > 0 && q->meetzero) q->credit += t.len;
      continue;
    }
    if (open) {
      group_phase[ngroups++] = cur_phase;
      group_start[ngroups] = (int32_t)nrel;
      open = false;
    }
    if (next >= n && q->nsched + q->fifo.size() == 0) break;
    if (++idle > max_idle) return bpsr::fail(BYTEPS_REDUCE_EARGS, "scheduler made no progress");
  }
  if (ngroups == 0) group_start[0] = 0;
  return ngroups;
}

int byteps_prophet_profile(const int64_t* tic_us, int32_t ngrad, int32_t* checkpoints,
                           double* backward_exec, int32_t cap) {
  if (!tic_us || !checkpoints || !backward_exec || ngrad < 1)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "null array or ngrad < 1");
  for (int32_t i = 0; i < ngrad; ++i)
    if (tic_us[i] < 0) return bpsr::fail(BYTEPS_REDUCE_EARGS, "tic of gradient %d < 0", i);
  // :129-135 running mean of the gaps, doubled
  double avg = 0;
  for (int32_t i = 1; i < ngrad; ++i) {
    const double x = std::fabs((double)(tic_us[i] - tic_us[i - 1]));
    avg = ((double)(i - 1) / i) * avg + (1.0 / i) * x;
  }
  avg *= 2;
  // :136-152
  std::vector<int32_t> cps{-1};
  std::deque<double> ex;
  for (int32_t i = 1; i < ngrad; ++i) {
    double diff = std::fabs((double)(tic_us[i] - tic_us[i - 1]));
    if (diff > avg) {
      diff /= 1000;
      if (ex.empty()) ex.push_back(std::fabs((double)(tic_us[i - 1] - tic_us[0])) / 1000);
      cps.push_back(i - 1);
      ex.push_front(diff);
    }
  }
  cps.push_back(ngrad - 1);
  if (ex.empty()) ex.push_back(std::fabs((double)(tic_us[ngrad - 1] - tic_us[0])) / 1000);
  ex.push_back(0);  // one entry per checkpoint (the last is never opened)
  if (cps.size() > (size_t)cap || ex.size() > (size_t)cap)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "cap %d < %zu checkpoints", cap, cps.size());
  if (cps.size() != ex.size())
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "internal: %zu checkpoints, %zu exec entries",
                      cps.size(), ex.size());
  for (size_t i = 0; i < cps.size(); ++i) {
    checkpoints[i] = cps[i];
    backward_exec[i] = ex[i];
  }
  return (int)cps.size();
}

int byteps_prophet_estimate_net_b(const int64_t* size, const int64_t* start_us,
                                  const int64_t* finish_us, int32_t n, double* net_b) {
  if (!size || !start_us || !finish_us || !net_b || n < 1)
    return bpsr::fail(BYTEPS_REDUCE_EARGS, "null array or n < 1");
  double best = -1;
  for (int32_t i = 0; i < n; ++i) {
    const int64_t t = finish_us[i] - start_us[i];
    if (t <= 0 || size[i] < 0) continue;
    const double mbps = (double)size[i] * 8.0 / (double)t;  // = possible_B / 125
    if (mbps > best) best = mbps;
  }
  if (best < 0) return bpsr::fail(BYTEPS_REDUCE_EARGS, "no push with finish > start");
  *net_b = best;
  return 0;
}

}  // extern "C"

namespace bpsr {
int prophet_poll(byteps_prophet_queue* q, byteps_prophet_task* out, bool* progressed) {
  std::lock_guard<std::mutex> g(q->mu);
  int32_t ph = 0;
  return q->poll(out, &ph, progressed) ? 1 : 0;
}

int prophet_add_many(byteps_prophet_queue* q, const byteps_prophet_task* t, size_t n) {
  std::lock_guard<std::mutex> g(q->mu);
  for (size_t i = 0; i < n; ++i)  // all or nothing
    if (const int rc = q->validate(t[i])) return rc;
  for (size_t i = 0; i < n; ++i) (void)q->add(t[i]);
  return 0;
}

size_t prophet_drain(byteps_prophet_queue* q, std::vector<byteps_prophet_task>* released) {
  std::lock_guard<std::mutex> g(q->mu);
  const size_t first = released->size();
  size_t group = first;  // first task of the open release group
  for (;;) {
    byteps_prophet_task t;
    int32_t ph = 0;
    bool prog = false;
    if (q->poll(&t, &ph, &prog)) {
      released->push_back(t);
      continue;
    }
    if (group != released->size()) {  // a group ended: report_finish, :367-369
      for (size_t i = group; i < released->size(); ++i)
        if ((*released)[i].len > 0 && q->meetzero) q->credit += (*released)[i].len;
      group = released->size();
      continue;
    }
    if (!prog) break;
  }
  return released->size() - first;
}
}  // namespace bpsr
