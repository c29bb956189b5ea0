/*
 * rs_batchio.h — host C-ABI of the RSCB batch file (librs_hip.so, host code
 * only; SURVEY §8(f) rank 2: the input producer's on-disk format).
 *
 * Replaces the hand-off of the reference's input producer
 * (algorithm/deep_learning/utils/dataset.py:36-65, create_criteo_dataset:
 * fillna -> MinMaxScaler -> LabelEncoder -> X[N, 13+26] float64 with the ids
 * packed as floats, which the Keras model casts to float32 — exact only below
 * 2^24 — and back to int32 in Embedding, layer/core.py:271) and of
 * features_dict (:69-75, vocab = nunique()+1).  An RSCB file holds the same
 * rows in the GPU path's layout: dense float32 [N, n_dense], label codes
 * int32/int64 [N, n_sparse], labels float32 [N] (each section one contiguous,
 * 4 KiB-aligned slab, so a batch is three DMA copies), plus the per-field
 * vocab sizes and one-hot offsets.  Status codes as in rs_capi.h.
 */
#ifndef RS_BATCHIO_H
#define RS_BATCHIO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Write n_rows rows (row-major host arrays).  Every id must lie in
 * [0, field_vocab[c]) (RS_ERR_ARG otherwise, nothing written);
 * field_offsets NULL = the running sum of field_vocab; labels may be NULL
 * (zeros).  id_bytes: 4 (int32) or 8 (int64).                              */
int rs_cb_write(const char* path, int64_t n_rows, int n_dense, int n_sparse,
                int id_bytes, const float* dense, const void* ids,
                const float* labels, const int64_t* field_vocab,
                const int64_t* field_offsets);
/* mmap an RSCB file; NULL on error (rs_last_error_string()).              */
void* rs_cb_open(const char* path);
int rs_cb_info(void* file, int64_t* n_rows, int* n_dense, int* n_sparse,
               int* id_bytes, int64_t* field_vocab, int64_t* field_offsets);
/* Copy rows [row0, row0+count) of each section into caller buffers (any may
 * be NULL) — pinned host buffers for the H2D stage; large slabs are copied
 * by up to 8 threads.                                                      */
int rs_cb_read(void* file, int64_t row0, int64_t count, float* dense,
               void* ids, float* labels);
void rs_cb_close(void* file);

#ifdef __cplusplus
}
#endif
#endif /* RS_BATCHIO_H */
