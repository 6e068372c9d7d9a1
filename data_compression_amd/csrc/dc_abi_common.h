// dc_abi_common.h -- shared helpers of the drop-in shims (libdc_huffman/nybble/small.so).
#pragma once
#include <stdio.h>
#include <stdlib.h>

#include "dc_gpu.h"
#include "dc_host.h"

// The reference reports misuse with assert() (abort). The void drop-in functions do the
// same on a HIP failure: they never fall back to CPU compute.
[[noreturn]] static inline void dc_die(const char *fn, int rc)
{
    fprintf(stderr, "%s: GPU path failed (status %d); no CPU fallback exists\n", fn, rc);
    abort();
}

#define DC_OR_DIE(fn, x) do { int _r = (x); if (_r) dc_die(fn, _r); } while (0)
