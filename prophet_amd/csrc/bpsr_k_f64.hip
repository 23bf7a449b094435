// Fold / batched kernels for one dtype family (see bpsr_kernels_impl.h).
#include "bpsr_kernels_impl.h"

BPSR_DEFINE_LAUNCHERS(f64, OpF64)
