/* C99 driver of the native Prophet scheduler (include/bpsr/prophet.h), built
 * by tests/test_abi.py with gcc against libbpsr.so: one iteration of the
 * 4-gradient hand trace (tests/test_prophet.py) through get_task polls, then
 * the same arrivals through byteps_prophet_release_groups.  Prints
 * "grad:phase" per release and "|" between groups. */
#include <stdio.h>
#include <string.h>

#include "bpsr/prophet.h"

int main(void) {
  const int32_t cps[3] = {-1, 1, 3};
  const double exec_[3] = {2, 5, 0};
  byteps_prophet_config cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.batch_size = 64;
  cfg.net_b = 1;
  cfg.credit = 150;
  cfg.checkpoints = cps;
  cfg.ncheckpoints = 3;
  cfg.backward_exec = exec_;
  byteps_prophet_queue* q = NULL;
  if (byteps_prophet_create(&cfg, &q)) return 2;
  byteps_prophet_task arr[4];
  for (int i = 0; i < 4; ++i) {
    memset(&arr[i], 0, sizeof(arr[i]));
    arr[i].grad = 3 - i;
    arr[i].len = 100;
    arr[i].total_partnum = 1;
    arr[i].scheduled = 1;
    arr[i].key = (uint64_t)(3 - i) << 16;
    arr[i].handle = 100 + i;
    if (byteps_prophet_add_task(q, &arr[i])) return 3;
  }
  for (int poll = 0; poll < 40; ++poll) {
    byteps_prophet_task t;
    int32_t ph = 0;
    const int rc = byteps_prophet_get_task(q, &t, &ph);
    if (rc < 0) return 4;
    if (rc == 1) {
      printf("%d:%d ", t.grad, ph);
      byteps_prophet_report_finish(q, t.len);
    }
  }
  printf("\n");
  byteps_prophet_task rel[4];
  int32_t start[5], phase[4];
  if (byteps_prophet_reset(q)) return 5;
  const int ng = byteps_prophet_release_groups(q, arr, 4, 1, 1, 1000, rel, start, phase);
  if (ng < 0) return 6;
  for (int g = 0; g < ng; ++g) {
    for (int i = start[g]; i < start[g + 1]; ++i) printf("%d:%d:%llu ", rel[i].grad, phase[g],
                                                          (unsigned long long)rel[i].handle);
    printf("| ");
  }
  printf("\n");
  byteps_prophet_destroy(q);
  /* pre-run profile: gaps of 100 us, 2,000 before gradient 3, 5,000 before 7 */
  int64_t tic[10];
  int64_t t = 1000000;
  for (int i = 9; i >= 0; --i) {
    tic[i] = t;
    if (i) t += i == 3 ? 2000 : i == 7 ? 5000 : 100;
  }
  int32_t pc[12];
  double pe[12];
  const int k = byteps_prophet_profile(tic, 10, pc, pe, 12);
  if (k < 0) return 7;
  for (int i = 0; i < k; ++i) printf("%d:%g ", pc[i], pe[i]);
  printf("\n");
  const int64_t sz[1] = {4096000}, st[1] = {0}, fi[1] = {3277};
  double nb = 0;
  if (byteps_prophet_estimate_net_b(sz, st, fi, 1, &nb)) return 8;
  printf("%.3f\n", nb);
  return 0;
}
