// Backward of the fused MAT decoder (token-on-lane tiles, mat_dec_ct.hip) as its own translation unit: EIGHT
// waves per workgroup over the one shared ~150 KB LDS tile (two waves per SIMD, two row tiles per wave at most).
// The 4-wave backward sat at 512 registers per wave (one wave per SIMD): every LDS / global latency and barrier of
// its ~20 phases per block was exposed.  With 8 waves each wave holds half the row tiles (<= 256 registers) and
// the second wave on each SIMD fills the first one's waits.  -DMDL_CT_BWD_NW=4 rebuilds the round-2 4-wave layout.
#ifndef MDL_CT_BWD_NW
#define MDL_CT_BWD_NW 8
#endif
#define MDL_NW MDL_CT_BWD_NW
#if MDL_CT_BWD_NW == 8
#define MDL_MAXRT 2
#endif
#define MDL_CT_BWD_TU
#include "mat_dec_ct.hip"
