// Fold / batched kernels for one dtype family (see bpsr_kernels_impl.h).
#include "bpsr_kernels_impl.h"

BPSR_DEFINE_LAUNCHERS(f16, OpF16)
