// mp4x native C API (CDNA4 / gfx950).
//
// One C ABI shared by every kernel translation unit and called from Python via
// ctypes (mp4x/ops/native.py).  All entry points are stream-ordered (no host
// synchronisation, no allocation) so they can be captured in hipGraphs.
// Return value: 0 on success, otherwise a hipError_t / MP4X_E* code.
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Element types — keep in sync with mp4x/operators.py DType.
enum mp4x_dtype {
  MP4X_F64 = 0, MP4X_F32 = 1, MP4X_I64 = 2, MP4X_I32 = 3, MP4X_I16 = 4, MP4X_I8 = 5,
  MP4X_BF16 = 6, MP4X_F16 = 7, MP4X_U8 = 8,
};

// Reduction operators — keep in sync with mp4x/operators.py OpCode.
// Reference table: /root/reference/src/main/java/com/fenbi/mp4j/operator/Operators.java:29-353
enum mp4x_op {
  MP4X_SUM = 0, MP4X_MAX = 1, MP4X_MIN = 2, MP4X_PROD = 3,
  MP4X_BAND = 4, MP4X_BOR = 5, MP4X_BXOR = 6,
  MP4X_FMAXLOC = 7, MP4X_FMINLOC = 8,   // f64 word: f32 value in hi 32 bits, int32 loc in lo 32 bits
  MP4X_IMAXLOC = 9, MP4X_IMINLOC = 10,  // i64 word: i32 value in hi 32 bits, int32 loc in lo 32 bits
  MP4X_FIRST = 11,                      // keep the first value (K8 map merge / dedupe-by-key; sparse only)
};

enum { MP4X_E_BADARG = 1001, MP4X_E_UNSUPPORTED = 1002,
       // latency fast path (mp4x_ipc_fast_allreduce): not launched, the caller takes the full path
       MP4X_E_FAILED_EARLIER = 1003,   // an IPC collective of this engine timed out earlier
       MP4X_E_CAPTURING = 1004,        // the stream is being captured into a hipGraph
       // a communicator's launch on a second stream inside ONE graph capture (the stream-order
       // guard cannot join a capture's forked streams: csrc/runtime/order.hip)
       MP4X_E_STREAM_SWITCH = 1005 };

#define MP4X_MAX_NIN 8

// ---------------------------------------------------------------- K1 / K1b / K2
// out[i] = op(...op(op(in[0][i], in[1][i]), in[2][i])..., in[nin-1][i])  for i < n.
// `out` may alias in[0] (the usual in-place accumulate).  nin in [1, MP4X_MAX_NIN]
// per launch; larger fan-in is chained by the caller.  16-bit floats accumulate in f32
// across the whole fan-in and round once.
int mp4x_reduce(int dtype, int op, void* out, const void* const* ins, int nin, int64_t n, void* stream);

// Same, but every input is the same buffer at a different element offset:
// in[k] = base + k * stride_elems.  Used after an all-to-all (p received chunks laid
// out contiguously) without building a pointer array.
int mp4x_reduce_strided(int dtype, int op, void* out, const void* base, int64_t stride_elems, int nin,
                        int64_t n, void* stream);

// out[i] = in[i] * scale (f32 / f64 / bf16 / f16), e.g. gradient averaging after a SUM.
int mp4x_scale(int dtype, void* out, const void* in, double scale, int64_t n, void* stream);

// ---------------------------------------------------------------- K3 segment copy
// Copy nseg byte segments in ONE launch: dst + dst_off[s] <- src + src_off[s], len[s] bytes.
// The three int64 tables live in DEVICE memory (3 * nseg entries: dst_off | src_off | len).
int mp4x_segment_copy(void* dst, const void* src, const int64_t* dev_table, int nseg, int64_t max_len,
                      void* stream);

// Row gather: out[i, :] = in[idx[i], :] for rows of `row_bytes` bytes.
int mp4x_gather_rows(void* out, const void* in, const int64_t* idx, int64_t nrows, int64_t row_bytes,
                     void* stream);

// ---------------------------------------------------------------- K6 codec (fp8 e4m3, OCP)
// Block-scaled quantisation: scale[b] = amax(block b) / 448, q = fp8(x / scale).
// block must be 256 (one wave, 4 elements per lane).  n must be a multiple of 4.
int mp4x_quant_fp8(int dtype_in, const void* in, int64_t n, uint8_t* q, float* scales, void* stream);
// out = dequant(q[0]) + ... + dequant(q[nin-1])  (f32 accumulate), optionally + out (accumulate=1).
// If q_out != NULL the f32 result is also re-quantised into (q_out, s_out).
int mp4x_dequant_reduce_fp8(int dtype_out, void* out, const uint8_t* const* qs, const float* const* scales,
                            int nin, int64_t n, int accumulate, uint8_t* q_out, float* s_out, void* stream);
int mp4x_dequant_fp8(int dtype_out, void* out, const uint8_t* q, const float* scales, int64_t n, void* stream);

// K6b lossless zero suppression.  table (device int64): elem_start[nchunk], elem_len[nchunk],
// blk_start[nchunk + 1] in 256-element blocks.  Encode: masks[4 * nblk], counts[nblk],
// offs[nblk + 1] (offs[nblk] = total non-zero words), vals (worst case n words).  Decode:
// the same masks / counts / vals (chunks concatenated) expanded into out per table.
size_t mp4x_zs_temp_bytes(int64_t nblk);
int mp4x_zs_encode(int elem_bytes, const void* in, const int64_t* table, int nchunk, int64_t nblk, uint64_t* masks,
                   int32_t* counts, int64_t* offs, void* vals, void* temp, size_t temp_bytes, void* stream);
int mp4x_zs_decode(int elem_bytes, const uint64_t* masks, const int32_t* counts, const void* vals,
                   const int64_t* table, int nchunk, int64_t nblk, void* out, int64_t* offs, void* temp,
                   size_t temp_bytes, void* stream);

// ---------------------------------------------------------------- K4 / K5 / K7 sparse
// Owner of each key: dest[i] = (uint64)key[i] % p.  hist[p] += counts (hist zeroed by caller).
int mp4x_key_owner(const int64_t* keys, int64_t n, int p, int32_t* dest, int32_t* hist, void* stream);
// Stable radix sort of (key, idx) pairs on bits [begin_bit, end_bit).
size_t mp4x_sort_pairs_temp_bytes(int64_t n, int key_is_i32);
int mp4x_sort_pairs_i64(const int64_t* keys_in, int64_t* keys_out, const int64_t* idx_in, int64_t* idx_out,
                        int64_t n, int begin_bit, int end_bit, void* temp, size_t temp_bytes, void* stream);
int mp4x_sort_pairs_i32key(const int32_t* keys_in, int32_t* keys_out, const int64_t* idx_in, int64_t* idx_out,
                           int64_t n, int begin_bit, int end_bit, void* temp, size_t temp_bytes, void* stream);
// Fused stable partition by owner ((uint64)key % p, p <= 2048): out_keys / out_vals (rows of
// row_bytes, 16-B aligned; vals may be NULL) in owner-major, input-stable order; out_perm
// (optional) = source row of every slot; counts[p] = rows per owner; range[2] (optional) = the
// smallest and largest key (0, 0 when n == 0).  Deterministic.
size_t mp4x_partition_pack_scratch_bytes(int64_t n, int p);
int mp4x_partition_pack(const int64_t* keys, const void* vals, int64_t n, int64_t row_bytes, int p,
                        int64_t* out_keys, void* out_vals, int64_t* out_perm, int64_t* counts, int64_t* range,
                        void* scratch, size_t scratch_bytes, void* stream);
// The two halves of mp4x_partition_pack (the same scratch between them): count -> counts[p],
// range[2]; scatter -> out_keys (key_stride 1: int64[n]; 2: the key half of 16-byte vectors),
// out_vals, out_perm.
int mp4x_partition_pack_count(const int64_t* keys, int64_t n, int p, int64_t* counts, int64_t* range, void* scratch,
                              size_t scratch_bytes, void* stream);
int mp4x_partition_pack_scatter(const int64_t* keys, const void* vals, int64_t n, int64_t row_bytes, int p,
                                int64_t* out_keys, int key_stride, void* out_vals, int64_t* out_perm, void* scratch,
                                size_t scratch_bytes, void* stream);
// Run-length encode a SORTED key array: starts[u] = first index of run u, *nruns (device int64).
size_t mp4x_rle_temp_bytes(int64_t n);
int mp4x_run_starts(const int64_t* sorted_keys, int64_t n, int64_t* starts, int64_t* nruns_dev,
                    int32_t* flags_scratch, void* temp, size_t temp_bytes, void* stream);
// Reduce-by-key over runs: for run u (rows perm[starts[u] .. starts[u+1])), out_vals[u, :] =
// op over those rows of `vals` (row length dim, dtype), in run order; out_keys[u] = key;
// out_count[u] = run length.  nruns is read from device memory.
int mp4x_segment_reduce_rows(int dtype, int op, const int64_t* sorted_keys, const int64_t* perm,
                             const int64_t* starts, const int64_t* nruns_dev, int64_t n, int64_t max_runs,
                             const void* vals, int64_t dim, int64_t* out_keys, void* out_vals, int32_t* out_count,
                             void* stream);

// ---------------------------------------------------------------- info
const char* mp4x_version(void);
int mp4x_device_count(void);

#ifdef __cplusplus
}
#endif
