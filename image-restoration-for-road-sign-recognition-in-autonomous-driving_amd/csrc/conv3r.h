// conv3r.h -- internal interface of the tap-reuse 3x3 conv (conv3r.hip),
// called from rr_igemm / rr_igemm_bnbwd (igemm.hip).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "igemm_epi.h"

// the column block BC the tap-reuse kernel would use for *d, 0 when it does
// not take the descriptor (bf16 3x3, square 8 / 16 / 32 maps, whole tiles)
int conv3r_bc(const rr_igemm_desc *d);
// rows of its BN statistics / BN-backward partial slabs (128-pixel blocks)
int conv3r_stat_blocks(const rr_igemm_desc *d);
// launch (a filled by igemm.hip's fill_args); returns an RR_* status
int conv3r_launch(const rr_igemm_desc *d, IgemmArgs &a, hipStream_t st);
// the kernel symbol for *d (static string)
const char *conv3r_name(const rr_igemm_desc *d);
