/* lz_diag.h -- measurement-only entry points of the DIAGNOSTIC build
 * (`make diag` -> lib/liblz_hip_diag.so; load it with LZ_HIP_LIB).  Nothing here
 * is in the shipped liblz_hip.so, and no solve uses it.
 *
 * Round-5 column-panel SpMM candidate (csrc/lz_panel.hip): parity-green, 4.3x
 * slower than lz_csr_spmm at C3 (profiles/r05e_panel_ab.log,
 * r05_pmc_spmm_panel_vs_seg.json); kept for its A/B (scripts/panel_ab.py, whose
 * panel_plan builds the plan below). */
#pragma once
#include "lz_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Candidate (round 5, measured against lz_csr_spmm at b = 16 fp64; DESIGN.md 4
 * SpMM "column panels"): Y = A X with X staged through LDS in 512-row panels
 * and row accumulators in registers, one 1024-thread block per 2048 rows, from
 * a once-per-operator plan of passes (scripts/panel_ab.py panel_plan builds
 * it): bp0[nblocks + 1] each block's pass range; per pass px0 (first X row of
 * its panel), pe0[npass + 1] (first entry, a multiple of 8), goff (136 uint16
 * per pass: the offsets of the block's 128 groups' entry lists, 129 used);
 * ev / ex the entries' values and (row slot << 9 | panel row) words.  X has nx
 * rows, row-major, ld = 16; Y n rows, ld = 16.  All arrays device. */
int lz_debug_spmm_panel(lz_handle *h, int64_t n, int64_t nx, const void *X, void *Y, int nblocks,
                        const int32_t *bp0, const int32_t *px0, const int32_t *pe0, const uint16_t *goff,
                        const void *ev, const uint16_t *ex);

#ifdef __cplusplus
}
#endif
