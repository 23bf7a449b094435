// Host-only error reporting shared by every C-ABI entry point (no HIP types,
// so host-only sources such as bpsr_prophet.cpp build with a plain C++
// compiler, e.g. under ThreadSanitizer in tests/test_prophet_native.py).
#pragma once

namespace bpsr {

// Thread-local message for byteps_reduce_last_error; returns `code`.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace bpsr
