// prims.h — device primitives behind the mtx_prefix_sum / hashgrid /
// scatter_reduce entry points (prefix_sum.py, hashgrid.py, reductions.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtx_core/field.h"

namespace mtxd {

size_t scan_workspace_bytes(uint64_t n);
// Device-wide u32 scan (single pass, decoupled look-back). in/out device.
int scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, int inclusive, void *ws, hipStream_t st);
// Hillis-Steele f32 scan in the reference's summation order; a and b are
// device ping-pong buffers (a holds the input); *result points at the one
// holding the output.
int scan_f32_hs(float *a, float *b, uint64_t n, float **result, hipStream_t st);
// the same from a read-only `in`; the result lands in `out` (tmp: n floats)
int scan_f32_hs_to(const float *in, float *out, float *tmp, uint64_t n, hipStream_t st);

size_t hashgrid_workspace_bytes(uint64_t n, uint32_t n_cells);
int hashgrid_build(const float *p, uint64_t n, uint32_t res, uint32_t n_cells, uint32_t *cell, uint32_t *cell_size,
                   uint32_t *cell_offset, uint32_t *sample_idx, void *ws, hipStream_t st);

// Stable group-by of n keys < n_keys (hash-grid machinery; workspace:
// hashgrid_workspace_bytes(n, n_keys)).
int group_by_u32(const uint32_t *keys, uint64_t n, uint32_t n_keys, uint32_t *key_size, uint32_t *key_offset,
                 uint32_t *order, void *ws, hipStream_t st);

// *bad (device word, zeroed by the caller) becomes non-zero if a key >= n_keys.
int keys_in_range(const uint32_t *keys, uint64_t n, uint32_t n_keys, uint32_t *bad, hipStream_t st);

// Stable sort permutation of n keys < 2^24 (hash-grid machinery).
size_t sort24_workspace_bytes(uint64_t n);
int sort24(const uint32_t *keys, uint64_t n, uint32_t *perm, void *ws, hipStream_t st);

size_t scatter_workspace_bytes(uint64_t n_target, uint64_t n_value);
int scatter_reduce_f32(int op, float *target, uint64_t n_target, const float *value, const uint32_t *index,
                       uint64_t n_value, void *ws, hipStream_t st);

// Radiance field (field.hip)
uint32_t field_frag_count(uint32_t n_hidden);
void field_prepack(const uint16_t *weights, uint32_t n_in, uint32_t n_hidden, uint16_t *frag);
// perm (optional): row i encodes query perm[i]; xcd_split: the blocks of one
// XCD take one contiguous eighth of the rows (rows grouped by region)
int field_encode(const mtx::FieldEncoding &e, const float4 *qp, const float4 *qd, const uint32_t *count,
                 uint32_t n_max, uint16_t *feat, hipStream_t st, const uint32_t *perm = nullptr, int xcd_split = 0,
                 int level_major = 0);
// Groups the cache queries by region (512 Morton cells of the field's box)
// on the device: perm[row] = query; cursor: a 32768-word workspace. No host sync.
void field_bucket_queries(const mtx::FieldEncoding &e, const float4 *qp, const uint32_t *count, uint32_t n_max,
                          uint32_t *cursor, uint32_t *perm, int n_cu, hipStream_t st);
// 24-bit Morton codes (8 bits per axis of the field's bounding box) of n queries
void field_morton_keys(const mtx::FieldEncoding &e, const float4 *qp, uint32_t n, uint32_t *keys, hipStream_t st);
// The NRC cache pass in one launch: encode + MLP + L_final[path] += T * out
// (qt: T.xyz, path bits in .w), rows in perm order.
size_t field_cache_fused_lds(uint32_t n_hidden);
int field_cache_fused(const mtx::FieldEncoding &e, const float4 *qp, const float4 *qd, const float4 *qt,
                      const uint32_t *count, uint32_t n_max, const uint32_t *perm, int xcd_split, const void *wfrag,
                      uint32_t n_hidden, float4 *L_final, int n_cu, hipStream_t st);
int field_mlp(const uint16_t *feat, const uint32_t *count, uint32_t n_max, const void *wfrag, uint32_t n_hidden,
              float *out, int n_cu, hipStream_t st);

// Radiance-field training (field_train.hip)
size_t field_train_lds(uint32_t n_hidden);
int field_train_launch(const uint16_t *feat, uint32_t n, const uint16_t *w16, uint32_t n_in, uint32_t n_hidden,
                       const float *target, float gscale, float *out, float *wave_loss, float *wpart, float *grad_w,
                       float *dfeat, uint32_t n_grid, hipStream_t st);
void field_encode_bwd_launch(const mtx::FieldEncoding &e, const float4 *qp, uint32_t n, const float *dfeat,
                             float *gtab, hipStream_t st);
void grad_check_launch(const float *g, uint64_t n, uint32_t *flag, hipStream_t st);
void adam_launch(float *p, float *m, float *v, const float *g, uint64_t n, float lr_t, float b1, float b2, float eps,
                 float inv_scale, const uint32_t *flag, uint16_t *tab16, uint64_t n_tab, uint16_t *w16,
                 hipStream_t st);
void half_to_float_launch(const uint16_t *h, uint64_t n, float *f, hipStream_t st);
void field_prepack_launch(const uint16_t *w16, uint32_t n_in, uint32_t n_hidden, uint16_t *frag, hipStream_t st);

}  // namespace mtxd
