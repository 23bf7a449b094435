// What the server group (bpsr_server_group.cpp) needs from a server instance
// beyond the C ABI of include/bpsr/server.h.  Not exported.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "bpsr/server.h"

namespace bpsr {

// byteps_server_push_async whose arrival takes position `pos` (>= 0) of its
// round's order: the group stamps one order per range-split key and every
// instance folds its piece in it (fused policy; the init round's store comes
// from the push at the last position).  pos < 0: the instance's arrival order.
int server_push_async_at(byteps_server* s, uint64_t key, int worker, const void* data,
                         size_t len, int dtype, int location, byteps_server_push_cb cb, void* ctx,
                         int pos);
// Would a push of `len` bytes of `dtype` to `key` be accepted (not failed, not
// declared with another length or dtype)?  0 or the error it would return.
int server_check_key(byteps_server* s, uint64_t key, size_t len, int dtype);
// Fail `key` on this instance as a failed fold would: every waiter and every
// later call on it gets `rc`.
void server_fail_key(byteps_server* s, uint64_t key, int rc);
// Has the key's init round completed on this instance (false: unknown key)?
// An init push is answered only once every worker's init push is in.
bool server_key_inited(byteps_server* s, uint64_t key);
// Does byteps_server_pull_into_async work on this instance (default engine,
// sync mode)?
bool server_pulls_async(const byteps_server* s);

}  // namespace bpsr
