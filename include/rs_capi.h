/*
 * rs_capi.h — C-ABI of the MI355X-native CTR forward path (librs_hip.so).
 *
 * This is the drop-in boundary that replaces the TF/Keras ops used by the
 * reference's embedding-lookup + feature-interaction forward path
 * (Hcyand/recommender_system, algorithm/deep_learning/...).  Every entry point
 * below cites the reference interface it replaces.  The Python host layer
 * (recommender_system_amd/layers.py, models.py) mirrors the reference's Keras
 * Layer/Model API on top of these functions; any other host (ctypes, cgo, JNI)
 * binds the same symbols.
 *
 * Conventions
 *  - All tensors are caller-owned DEVICE pointers (HBM), row-major, contiguous
 *    unless a *_stride argument says otherwise (strides are in ELEMENTS).
 *  - Sizes are int64_t; small shape parameters are int.
 *  - Every function is stream-ordered on `stream` (a hipStream_t passed as
 *    void*; NULL = the legacy default stream), never allocates, never
 *    synchronises, and is safe to capture into a hipGraph.
 *  - Return value: RS_OK (0) or a negative rs_status; the message for the last
 *    failure on the calling thread is available from rs_last_error_string().
 *  - Sparse ids: `id_kind` selects int32 / int64 / float32.  float32 ids follow
 *    the reference's packed input X[B,39] (model/deepFM.py:24), where Keras'
 *    Embedding casts float ids to int32 by truncation.  An id outside
 *    [0, vocab_c) is an error in the reference (TF InvalidArgumentError on CPU);
 *    here the kernel reads a zero row instead and sets *err_flag = 1 (if
 *    err_flag != NULL), which the host layer turns into IndexError.
 */
#ifndef RS_CAPI_H
#define RS_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* rs_stream_t; /* hipStream_t */

enum rs_status {
  RS_OK = 0,
  RS_ERR_ARG = -1,         /* bad shape / null pointer / unsupported combination */
  RS_ERR_HIP = -2,         /* HIP launch or runtime error */
  RS_ERR_UNSUPPORTED = -3  /* valid request, no kernel for it in this build */
};

enum rs_id_kind { RS_ID_I32 = 0, RS_ID_I64 = 1, RS_ID_F32 = 2 };

enum rs_act {
  RS_ACT_NONE = 0,
  RS_ACT_RELU = 1,
  RS_ACT_PRELU = 2,   /* max(0,x) + alpha*min(0,x); alpha per output column  */
  RS_ACT_SIGMOID = 3
};

/* Bits of the device error flag (int, caller-owned, zero it before use):
 * kernels OR these in; the host layer raises IndexError for RS_FLAG_BAD_ID
 * (TF's InvalidArgumentError on an out-of-range Embedding id) and RSError for
 * any other bit. */
enum rs_flag {
  RS_FLAG_BAD_ID = 1, /* an id outside [0, vocab) (its row read as zeros)               */
  RS_FLAG_LAYOUT = 2, /* field row ranges overlap or decrease where a kernel needs the
                         concatenated-table layout (offset_c + vocab_c <= offset_{c+1}) */
  RS_FLAG_TIMEOUT = 4 /* a bounded in-kernel wait (a workgroup-internal hand-off) gave up:
                         a kernel logic error — the launch's outputs are invalid and the
                         host layer raises RSError instead of returning them               */
};

/* Runtime tuning options (host side, read when a kernel is launched, so a
 * captured hipGraph keeps the value it was captured with).  Options are
 * THREAD-LOCAL: rs_set_option changes only the launches made by the calling
 * host thread, every new thread starts from the defaults — no process-wide
 * mutable state, so concurrent callers on different threads stay reentrant
 * (SURVEY 8(b)).  They select between measured kernel forms for A/B work;
 * results agree within the parity tolerance whatever the setting. */
enum rs_option {
  RS_OPT_EMBED_FM_KERNEL = 0, /* rs_embed_fm_fwd kernel (id inputs, no x_out): 0 = MFMA K-split,
                                 1 = VALU/DPP persistent 8-sample tiles, 2 / 3 = MFMA persistent
                                 16-sample tiles (2 / 1 resident per CU); shapes a kernel does
                                 not cover run the K-split one.  See DESIGN.md 4.1                */
  RS_OPT_MLP_UNROLL = 1,      /* fused MLP towers (rs_mlp_fwd, rs_deepfm_fwd, rs_dcn_fwd): 1 (the
                                 default) = the k-group loop of the common layer widths fully
                                 unrolled (no loop-head wait on the weight ring), 0 = the looped
                                 form.  See DESIGN.md 4.5                                         */
  RS_OPT_DEEPFM_KERNEL = 2,   /* rs_deepfm_fwd_hm at the Criteo shape (k 16, 26 fields, 256-unit
                                 first layer): 0 (the default) = split wave roles (loaders +
                                 layer-0 compute waves, deepfm_ws), 1 = one role per wave (gather
                                 + FM, then the tower), 2 / 3 = every wave gathers two fields and
                                 computes one layer-0 tile, split-K tower tail (deepfm_all; a
                                 weight ring 3 / 4 k-groups deep).  See DESIGN.md 4.5            */
  RS_OPT_DIN_KERNEL = 3,      /* rs_din_attention_ids_fwd at the reference's (80, 40) widths: 0
                                 (the default) = one launch (scores + softmax + pool, din_fused),
                                 1 = two launches (din_scores, din_pool).  See DESIGN.md 4.4     */
  RS_OPT_PEER_FENCES = 4,     /* the peer-mapped exchange's ordering (rs_peer_a2a, rs_peer_gather_a2a,
                                 rs_shard_fm_pipe_peer): 0 (the default) = lean — write-through
                                 data stores, relaxed counts, write-through flags, no L2
                                 maintenance; 1 = a system-scope release / acquire fence around
                                 every count and flag.  See DESIGN.md 4.6                        */
  RS_OPT_CROSS_KERNEL = 5,    /* rs_embed_cross_fwd_hm / rs_dcn_fwd_hm (k 16, <= 32 fields, <= 16
                                 CrossNet B columns): 0
                                 (the default) = the contraction from the gathered registers as
                                 the rows land; 1 = the staged-tile contraction after the gather
                                 (bit-identical to rs_embed_cross_fwd).  See DESIGN.md 4.2       */
  RS_OPT_COUNT = 6
};

/* ------------------------------------------- peer-mapped exchange (§8(e))
 * An equal-split all-to-all for the sharded lookup's fixed-size record
 * exchanges without RCCL (csrc/peer.hip, sharded.py PeerExchange): every rank
 * owns one mailbox (rs_peer_alloc: uncached device memory, zeroed) of
 * rs_peer_mailbox_bytes(world, block_bytes) bytes = [world][block_bytes] data
 * + step flags, exports it (rs_peer_ipc_handle: a 64-byte hipIpcMemHandle_t)
 * and maps every peer's (rs_peer_ipc_open).  rs_peer_a2a is ONE launch per
 * exchange: rank `rank` writes block p of `send` into rank p's mailbox at
 * data[rank] once p has flagged its mailbox free for the step, flags it, and
 * the launch ends when every rank's block of the step is in its own mailbox.
 * mailboxes: device array [world] of every rank's mailbox base as seen by
 * this process (its own at [rank]); state: rs_peer_state_bytes() of zeroed
 * device memory, private to this rank and exchange (the step counter lives
 * there: graph-capturable).  Kernels that read the received data must run on
 * `stream` after the call and before the next rs_peer_a2a of the same
 * mailbox.  Bounded waits (spin_limit polls): a timeout sets RS_FLAG_TIMEOUT
 * in *err_flag.  block_bytes % 16 == 0, world <= 64, chunks * world <= 1024.
 * No reference counterpart (the reference has no distributed code).     */
int64_t rs_peer_state_bytes(void);
int64_t rs_peer_mailbox_bytes(int world, int64_t block_bytes);
int rs_peer_alloc(int64_t bytes, void** ptr);
int rs_peer_free(void* ptr);
int rs_peer_ipc_handle(void* ptr, void* handle64);
int rs_peer_ipc_open(const void* handle64, void** ptr);
int rs_peer_ipc_close(void* ptr);
int rs_peer_a2a(const void* send, int64_t block_bytes, void* const* mailboxes,
                int rank, int world, void* state, int chunks,
                int64_t spin_limit, int* err_flag, rs_stream_t stream);
/* The owner's row service fused with the row exchange (config 5): block p
 * for rank p is gathered on the fly — for every word i of ids[p][0..nw) the
 * 64-B row table[ids[p][i]] of the local shard (k = 16; -1 = a zero row, any
 * other id outside [0, n_rows) a zero row + RS_FLAG_BAD_ID) — and written
 * straight into rank p's mailbox (block_bytes = nw * 64); the same flags,
 * waits and state as rs_peer_a2a.  Replaces rs_gather_rows + the row
 * all-to-all of sharded.py ShardedDeepFM.                                 */
int rs_peer_gather_a2a(const int32_t* ids, int64_t nw, const float* table,
                       int64_t n_rows, int k, void* const* mailboxes, int rank,
                       int world, void* state, int chunks, int64_t spin_limit,
                       int* err_flag, rs_stream_t stream);

/* ------------------------------------------------------------------ meta */
const char* rs_version(void);
const char* rs_last_error_string(void);
/* Set option `option` to `value`; returns the previous value, or -1 for an
 * unknown option / out-of-range value (then nothing changes). */
int rs_set_option(int option, int value);
/* Current value of `option`, or -1 for an unknown option. */
int rs_get_option(int option);
/* Diagnostic (no reference counterpart): launch an empty kernel of `grid`
 * workgroups x `block` threads on `stream`.  bench.py replays it from a
 * hipGraph to record the box's dependent-launch slot time beside its
 * numbers. */
int rs_diag_empty(int grid, int block, rs_stream_t stream);
/* rs_diag_wave_slots: every wave's HW_ID register (bits 3:0 wave slot, 5:4
 * SIMD, 11:8 CU, 12 SH, 15:13 SE) into out[grid * block / 64], lds_bytes of
 * dynamic LDS per workgroup — how a workgroup's waves spread over the SIMDs. */
int rs_diag_wave_slots(int grid, int block, int lds_bytes, uint32_t* out, rs_stream_t stream);
/* rs_diag_mfma_chain: every wave issues n v_mfma_f32_16x16x4_f32 as `chains`
 * (1, 2, 4) independent accumulation chains; cyc[3 wave + {0, 1, 2}] = its
 * start / end s_memtime and its HW_ID (SIMD in bits 5:4), so the host can time
 * each SIMD's window from its first wave's start to its last wave's end. */
int rs_diag_mfma_chain(int grid, int block, int n, int chains, unsigned long long* cyc, float* sink,
                       rs_stream_t stream);
/* rs_diag_icache: 2048 FMAs per wave as a loop (unroll 0) or straight-line
 * code (unroll 1), run twice in one launch; cyc[2 wave + pass] = cycles.     */
int rs_diag_icache(int grid, int block, int unroll, unsigned long long* cyc, float* sink, rs_stream_t stream);

/* --------------------------------------------------------- embedding (a3)
 * Replaces EmbedLayer.call (layer/core.py:273-280) + the dense/sparse concat of
 * DeepFM.call / DCN.call (model/deepFM.py:24-26, model/dcn.py:25-27):
 *   out[b, 0:nd]               = dense[b, 0:nd]
 *   out[b, nd + c*k + j]       = table[field_offsets[c] + id(b,c), j]
 * One contiguous table holds every field's Keras `Embedding` matrix stacked
 * (field c occupies rows [field_offsets[c], field_offsets[c]+field_vocab[c])).
 * nd may be 0 (dense may then be NULL): the result is EmbedLayer's [B, F*k].
 * field_offsets / field_vocab are device int64[F].                          */
int rs_embed_gather(const void* ids, int id_kind, int64_t id_stride,
                    const float* dense, int64_t dense_stride, int nd,
                    const float* table, const int64_t* field_offsets,
                    const int64_t* field_vocab, int n_fields, int k,
                    float* out, int64_t out_stride, int64_t batch,
                    int* err_flag, rs_stream_t stream);

/* ---------------------------------------------------- FM second order (a5)
 * FMLayer.call (layer/interaction.py:106-114) on x = [dense | emb] with
 * d = nd + F*k, weights w0:(1,), w1:(d,1), v:(d,kfm):
 *   y[b] = x@w1 + w0 + 0.5*sum_f((x@v)_f^2 - (x^2 @ v^2)_f)
 * The kernels consume a packed weight image built once per weight set by
 * rs_fm_prepare (MFMA operand order + per-row squared norms of v); query its
 * size in floats with rs_fm_prepared_size.                                   */
int64_t rs_fm_prepared_size(int nd, int n_fields, int k, int kfm);
int rs_fm_prepare(const float* w1, const float* v, int nd, int n_fields, int k,
                  int kfm, float* prepared, rs_stream_t stream);

/* Fused EmbedLayer + concat + FMLayer (the headline kernel; DeepFM semantics,
 * model/deepFM.py:24-28).  logit[b] = FMLayer(x)[b]; if x_out != NULL the
 * concatenated x[B,d] (row stride d) is also written for the DNN tower.      */
int rs_embed_fm_fwd(const void* ids, int id_kind, int64_t id_stride,
                    const float* dense, int64_t dense_stride, int nd,
                    const float* table, const int64_t* field_offsets,
                    const int64_t* field_vocab, int n_fields, int k,
                    const float* prepared, const float* w0, int kfm,
                    float* logit, float* x_out, int64_t batch, int* err_flag,
                    rs_stream_t stream);
/* The same with the field metadata also given on the HOST (read at call
 * time, copied into the launch: graph capture keeps the values of the
 * capturing call).  For n_fields <= 32 and batch <= 8192 the kernel then
 * reads (offset, vocab) through scalar kernel-argument loads and each wave
 * loads its own fields' ids — no workgroup id tile, no barrier; otherwise
 * (or with a kernel option other than 0 set) it is rs_embed_fm_fwd.  The
 * host arrays must equal the device ones.                                    */
int rs_embed_fm_fwd_hm(const void* ids, int id_kind, int64_t id_stride,
                       const float* dense, int64_t dense_stride, int nd,
                       const float* table, const int64_t* field_offsets,
                       const int64_t* field_vocab,
                       const int64_t* field_offsets_host,
                       const int64_t* field_vocab_host, int n_fields, int k,
                       const float* prepared, const float* w0, int kfm,
                       float* logit, float* x_out, int64_t batch, int* err_flag,
                       rs_stream_t stream);

/* FMLayer on an arbitrary dense x[B,n] (layer/interaction.py:106-114), e.g.
 * the FM model's one-hot input (model/fm.py:19-23).  `prepared` comes from
 * rs_fm_prepare(w1, v, n, 0, 0, kfm, ...).                                   */
int rs_fm_fwd(const float* x, int64_t x_stride, int n, const float* prepared,
              const float* w0, int kfm, float* logit, int64_t batch,
              rs_stream_t stream);

/* FM model on the compact form of its one-hot input (model/fm.py:19-23 with
 * utils/dataset.py:47-48): x = [dense(nd) | onehot], where the one-hot block
 * has exactly one 1 per field at column nd + field_offsets[c] + id(b,c).
 * Gathers rows of v and w1 instead of multiplying by zeros.                  */
int rs_fm_onehot_fwd(const void* ids, int id_kind, int64_t id_stride,
                     const float* dense, int64_t dense_stride, int nd,
                     const int64_t* field_offsets, const int64_t* field_vocab,
                     int n_fields, const float* w1, const float* w0,
                     const float* v, int kfm, float* logit, int64_t batch,
                     int* err_flag, rs_stream_t stream);

/* ------------------------------------------------------ DCN CrossNet (a9)
 * CrossLayer.call (layer/interaction.py:75-83):
 *   x_{l+1} = x0 * (x_l^T w_l) + b_l + x_l,  l = 0..L-1,  out = x_L
 * w, b: [L, d] (Keras shapes (d,1) each, stacked).  The L contractions
 * x0^T w_l run on fp32 MFMA; `prepared` (rs_cross_prepared_size floats) holds
 * the packed weights and the sample-independent bias terms.                  */
int64_t rs_cross_prepared_size(int d, int n_layers);
int rs_cross_prepare(const float* w, const float* b, int d, int n_layers,
                     float* prepared, rs_stream_t stream);
int rs_cross_fwd(const float* x0, int64_t x_stride, int d, int n_layers,
                 const float* prepared, float* out, int64_t out_stride,
                 int64_t batch, rs_stream_t stream);

/* Fused DCN input + CrossNet: x0 = [dense | EmbedLayer(ids)] (model/dcn.py:
 * 24-27, layer/core.py:273-280) is assembled in LDS — never written to HBM —
 * and out = CrossLayer(x0) (layer/interaction.py:75-83).  Gather arguments as
 * rs_embed_gather; prepared from rs_cross_prepare(d = nd + F*k).  k % 4 == 0,
 * 1..128 fields, d <= 1600.  Out-of-range ids set *err_flag, rows read 0.    */
int rs_embed_cross_fwd(const void* ids, int id_kind, int64_t id_stride,
                       const float* dense, int64_t dense_stride, int nd,
                       const float* table, const int64_t* field_offsets,
                       const int64_t* field_vocab, int n_fields, int k,
                       int n_layers, const float* prepared, float* out,
                       int64_t out_stride, int64_t batch, int* err_flag,
                       rs_stream_t stream);
/* The same with the fields' (offset, vocab) also on the host: at k = 16 and
 * <= 32 fields they travel as kernel arguments and the rows come in through
 * the headline kernel's front end (per-wave field ids, no id tile; DESIGN.md
 * 4.2); otherwise identical to rs_embed_cross_fwd.  Bit-identical outputs. */
int rs_embed_cross_fwd_hm(const void* ids, int id_kind, int64_t id_stride,
                          const float* dense, int64_t dense_stride, int nd,
                          const float* table, const int64_t* field_offsets,
                          const int64_t* field_vocab,
                          const int64_t* field_offsets_host,
                          const int64_t* field_vocab_host, int n_fields, int k,
                          int n_layers, const float* prepared, float* out,
                          int64_t out_stride, int64_t batch, int* err_flag,
                          rs_stream_t stream);

/* Fused DCN forward (model/dcn.py:24-34) in one launch: x0 in LDS, CrossNet
 * folded into its contraction, the DNN tower on the same tile, head
 * sigmoid(Dense1([x_L | dnn])).  cross_prepared: rs_cross_prepare over
 * n_cross + 1 columns — w_0..w_{L-1} then the output Dense's cross half
 * w_o[:d] (bias row 0) — so the cross branch's logit is alpha_L (x0.w_o) +
 * beta_L.w_o without forming x_L.  mlp_prepared: rs_mlp_prepare of the DNN
 * hidden layers plus ONE folded last layer (W_last w_o[d:], b_last w_o[d:] +
 * b_o), dims[n_layers] == 1, no input permutation.  rs_dcn_fused_ok: shape
 * supported (k % 4 == 0, 1..128 fields, n_cross <= 31).                    */
int rs_dcn_fused_ok(int nd, int n_fields, int k, int n_cross, int n_layers,
                    const int* dims);
int rs_dcn_fwd(const void* ids, int id_kind, int64_t id_stride,
               const float* dense, int64_t dense_stride, int nd,
               const float* table, const int64_t* field_offsets,
               const int64_t* field_vocab, int n_fields, int k, int n_cross,
               const float* cross_prepared, int n_layers, const int* dims,
               const int* acts, const float* mlp_prepared, float* out,
               int64_t batch, int* err_flag, rs_stream_t stream);
/* rs_dcn_fwd with host field metadata (kernel-argument front end, as
 * rs_embed_cross_fwd_hm).  Bit-identical outputs. */
int rs_dcn_fwd_hm(const void* ids, int id_kind, int64_t id_stride,
                  const float* dense, int64_t dense_stride, int nd,
                  const float* table, const int64_t* field_offsets,
                  const int64_t* field_vocab, const int64_t* field_offsets_host,
                  const int64_t* field_vocab_host, int n_fields, int k,
                  int n_cross, const float* cross_prepared, int n_layers,
                  const int* dims, const int* acts, const float* mlp_prepared,
                  float* out, int64_t batch, int* err_flag, rs_stream_t stream);

/* ----------------------------------------------- PNN inner product (a11)
 * InnerProductLayer.call (layer/interaction.py:170-183) on e[B,F,k]:
 *   out[b,p] = <e[b,i_p,:], e[b,j_p,:]>, pairs (i<j) in row-major order.
 * out row stride is out_stride (>= F(F-1)/2).                               */
int rs_inner_product_fwd(const float* emb, int n_fields, int k, float* out,
                         int64_t out_stride, int64_t batch, rs_stream_t stream);

/* Fused gather + flatten + inner product: writes the PNN DNN input
 * out[b] = [flat_emb (F*k) | inner (F(F-1)/2)] (model/pnn.py:34-41).       */
int rs_embed_inner_fwd(const void* ids, int id_kind, int64_t id_stride,
                       const float* table, const int64_t* field_offsets,
                       const int64_t* field_vocab, int n_fields, int k,
                       float* out, int64_t out_stride, int64_t batch,
                       int* err_flag, rs_stream_t stream);
/* rs_embed_inner_fwd with host field metadata (kernel-argument front end at
 * k = 16, <= 32 fields).  Bit-identical outputs. */
int rs_embed_inner_fwd_hm(const void* ids, int id_kind, int64_t id_stride,
                          const float* table, const int64_t* field_offsets,
                          const int64_t* field_vocab,
                          const int64_t* field_offsets_host,
                          const int64_t* field_vocab_host, int n_fields, int k,
                          float* out, int64_t out_stride, int64_t batch,
                          int* err_flag, rs_stream_t stream);

/* OuterProductLayer (layer/interaction.py:186-215): out[b,p] =
 * sum_{a,j} e[b,row_p,j] W[a,p,j] e[b,col_p,a] with W the Keras weight
 * [k, P, k], pairs in the reference's row-major i<j order.  rs_outer_prepare
 * packs W into per-lane MFMA fragments (rs_outer_prepared_size floats; k in
 * {4,8,16,32,64}, 2..64 fields).  rs_outer_product_fwd: emb [B,F,k] -> out
 * [B,P].  rs_embed_product_fwd: PNN's DNN input (model/pnn.py:32-48) from ids
 * in one launch — out[b] = [flat_emb (F*k) | inner (P, if inner) | outer (P,
 * if outer_prepared)]; mode 'inner' / 'outer' / 'both'.                      */
int64_t rs_outer_prepared_size(int n_fields, int k);
int rs_outer_prepare(const float* W, int n_fields, int k, float* prepared,
                     rs_stream_t stream);
int rs_outer_product_fwd(const float* emb, int n_fields, int k,
                         const float* outer_prepared, float* out,
                         int64_t out_stride, int64_t batch, rs_stream_t stream);
int rs_embed_product_fwd(const void* ids, int id_kind, int64_t id_stride,
                         const float* table, const int64_t* field_offsets,
                         const int64_t* field_vocab, int n_fields, int k,
                         int inner, const float* outer_prepared, float* out,
                         int64_t out_stride, int64_t batch, int* err_flag,
                         rs_stream_t stream);
/* rs_embed_product_fwd with host field metadata (as rs_embed_inner_fwd_hm). */
int rs_embed_product_fwd_hm(const void* ids, int id_kind, int64_t id_stride,
                            const float* table, const int64_t* field_offsets,
                            const int64_t* field_vocab,
                            const int64_t* field_offsets_host,
                            const int64_t* field_vocab_host, int n_fields, int k,
                            int inner, const float* outer_prepared, float* out,
                            int64_t out_stride, int64_t batch, int* err_flag,
                            rs_stream_t stream);

/* ---------------------------------------------- DIN attention unit (a13)
 * Attention.call (layer/interaction.py:369-406), 'prelu' mode:
 *   e_t   = [q, key_t, q-key_t, q*key_t]                         (4k)
 *   h1_t  = PReLU_{alpha1[t]}(e_t @ W1 + b1)                     (H1)
 *   h2_t  = PReLU_{alpha2[t]}(h1_t @ W2 + b2)                    (H2)
 *   s_t   = h2_t @ w3 + b3;  s_t = -4294967296 where mask[b,t]==0
 *   out   = softmax_t(s) @ value                                 (k)
 * W1 [4k,H1], W2 [H1,H2], w3 [H2], alpha1 [T,H1], alpha2 [T,H2] (Keras
 * PReLU inside Dense on a 3-D input: alpha shape input_shape[1:]).
 * `mask` is float [B,T] (0 = padded).  Supported: k in {4,8,16,32},
 * H1,H2 <= 128.                                                              */
int rs_din_attention_fwd(const float* query, const float* keys,
                         const float* values, const float* mask, int T, int k,
                         const float* W1, const float* b1, const float* alpha1,
                         int H1, const float* W2, const float* b2,
                         const float* alpha2, int H2, const float* w3,
                         const float* b3, float* out, int64_t batch,
                         rs_stream_t stream);

/* Attention.call 'dice' mode (layer/interaction.py:363-364, 410-425): the
 * activation stack is n_dice Dice layers applied to e_t (no Dense), then
 * Dense(1).  Dice at inference: xhat=(x-mean)/sqrt(var+eps), p=sigmoid(xhat),
 * y = alpha*(1-p)*x + p*x; per-layer mean/var/alpha are [n_dice, 4k].        */
int rs_din_attention_dice_fwd(const float* query, const float* keys,
                              const float* values, const float* mask, int T,
                              int k, int n_dice, const float* dice_alpha,
                              const float* dice_mean, const float* dice_var,
                              float dice_eps, const float* w_out,
                              const float* b_out, float* out, int64_t batch,
                              rs_stream_t stream);

/* Attention.call 'prelu' at any depth (layer/interaction.py:355-406 with
 * len(hidden_units) = n_layers, any H, k <= 64 or larger): e = [q, key_t,
 * q-key_t, q*key_t] per (b, t) row, Dense(hidden[l], PReLU()) with alpha
 * [T, hidden[l]] as fp32 MFMA GEMMs over the B*T rows, Dense(1), masked
 * softmax, weighted sum of the values.  W[l] (in, out) Keras orientation,
 * b[l] [hidden[l]], alpha[l] [T, hidden[l]] (device pointers in host
 * arrays).  workspace: rs_din_attention_gen_workspace_size bytes (device).   */
int64_t rs_din_attention_gen_workspace_size(int64_t batch, int T, int k,
                                            int n_layers, const int* hidden);
int rs_din_attention_gen_fwd(const float* query, const float* keys,
                             const float* values, const float* mask, int T,
                             int k, int n_layers, const int* hidden,
                             const float* const* W, const float* const* b,
                             const float* const* alpha, const float* w_out,
                             const float* b_out, float* out, int64_t batch,
                             void* workspace, int64_t workspace_bytes,
                             rs_stream_t stream);

/* DIN attention straight from behaviour ids (model/din.py:56-80 + Attention
 * 'prelu', layer/interaction.py:355-406): key = value = table[hist[b,t]],
 * query = table[cand[b]], mask = hist != 0.  At the reference's (80, 40)
 * widths ONE launch (din_fused: every position's PReLU alphas and W2 staged
 * once per workgroup of 8 samples, layer 1 regrouped per sample as
 * q(Wq+Wd) + key(Wk-Wd+diag(q)Wp), per-tile online-softmax partials merged
 * per sample — the scores never reach HBM); other widths, or
 * RS_OPT_DIN_KERNEL 1, two launches (scores, then the masked softmax pool).
 * prepared: rs_din_prepare (k in {4,8,16}, H1 <= 128, H2 <= 64); scores: a
 * caller-owned [B, T] fp32 workspace (untouched by the one-launch form);
 * out [B, k] with rows out_stride
 * floats apart (>= k: DIN.call writes straight into its concat).  T <= 1024.
 * OOR ids set *err_flag.                                                   */
int64_t rs_din_prepared_size(int T, int k, int H1, int H2);
int rs_din_prepare(const float* W1, const float* b1, const float* alpha1,
                   int H1, const float* W2, const float* b2,
                   const float* alpha2, int H2, const float* w3,
                   const float* b3, int T, int k, float* prepared,
                   rs_stream_t stream);
int rs_din_attention_ids_fwd(const void* hist, int id_kind, int64_t hist_stride,
                             const void* cand, int64_t cand_stride, int T,
                             int k, const float* table, int64_t vocab, int H1,
                             int H2, const float* prepared, float* scores,
                             float* out, int64_t out_stride, int64_t batch,
                             int* err_flag, rs_stream_t stream);
/* ... and the candidate rows table[cand] into cand_out [B, k] (rows
 * cand_out_stride floats apart; an out-of-range id writes a zero row and sets
 * *err_flag), the copy DIN.call concatenates beside the pooled rows
 * (model/din.py:78-79,84-85): the same launch, no separate candidate gather.   */
int rs_din_attention_ids_cand_fwd(const void* hist, int id_kind,
                                  int64_t hist_stride, const void* cand,
                                  int64_t cand_stride, int T, int k,
                                  const float* table, int64_t vocab, int H1,
                                  int H2, const float* prepared, float* scores,
                                  float* out, int64_t out_stride,
                                  float* cand_out, int64_t cand_out_stride,
                                  int64_t batch, int* err_flag,
                                  rs_stream_t stream);

/* DIN.call (model/din.py:56-95) in ONE launch: the attention unit of
 * rs_din_attention_ids_cand_fwd, then BatchNormalization (in_scale / in_shift,
 * as rs_mlp_affine_fwd) + the PReLU tower + Dense(1, sigmoid) of
 * rs_mlp_affine_pieces_fwd over the input [pooled (k) | cand rows (k) |
 * pieces] — the pieces must cover columns 2k .. dims[0]-1 (in_cols >= 2k) —
 * writing y [B] (rows y_stride apart).  Bit-identical to those two launches.
 * pooled (optional, rows pooled_stride apart) also receives the attention
 * output.  rs_din_forward_ids_supported: 1 when the shape takes the fused
 * launch (the reference's (80, 40) attention, a 256-unit first layer and the
 * 128 -> 64 -> 1 tail, dims[0] <= 64), else 0 (the caller keeps two launches).
 * Replaces DIN.call's attention + concat + bn + dense_layer + out_layer. */
int rs_din_forward_ids_supported(int T, int k, int H1, int H2, int n_layers,
                                 const int* dims);
int rs_din_forward_ids(const void* hist, int id_kind, int64_t hist_stride,
                       const void* cand, int64_t cand_stride, int T, int k,
                       const float* table, int64_t vocab, int H1, int H2,
                       const float* att_prepared, float* pooled,
                       int64_t pooled_stride, const float* in_scale,
                       const float* in_shift, int n_layers, const int* dims,
                       const int* acts, const float* tower_prepared, float* y,
                       int64_t y_stride, int n_pieces, const int* widths,
                       const int* in_cols, const int* kinds,
                       const void* const* srcs, const int64_t* src_strides,
                       const float* const* tables, const int64_t* vocabs,
                       int64_t batch, int* err_flag, rs_stream_t stream);

/* ------------------------------------------------ concat pieces (a15, a3)
 * One launch for the concat pieces that live in different tables: piece p
 * writes widths[p] columns of out [B, *] (rows out_stride floats apart)
 * starting at out_cols[p].  kinds[p] = RS_ID_* : a sparse feature, one id
 * per sample (srcs[p], src_strides[p] elements apart) looked up in
 * tables[p] [vocabs[p], widths[p]] (Keras Embedding; an out-of-range id
 * writes a zero row and sets *err_flag); kinds[p] = -1: dense fp32 values
 * [B, widths[p]] copied as they are.  DIN.call's other sparse embeddings and
 * dense features (model/din.py:64-69,84-85).  1..16 pieces.                      */
int rs_concat_pieces(int n_pieces, const int* widths, const int* out_cols,
                     const int* kinds, const void* const* srcs,
                     const int64_t* src_strides, const float* const* tables,
                     const int64_t* vocabs, float* out, int64_t out_stride,
                     int64_t batch, int* err_flag, rs_stream_t stream);

/* --------------------------------------------------- dense tower (a7, a15)
 * Keras Dense: y = act(x @ W + bias), W:[K,N] (Keras (in,out) orientation),
 * fp32 MFMA.  alpha: per-column PReLU slope (RS_ACT_PRELU only).            */
int rs_dense_fwd(const float* x, int64_t x_stride, const float* W,
                 const float* bias, const float* alpha, int act, float* y,
                 int64_t y_stride, int64_t M, int K, int N, rs_stream_t stream);

/* ------------------------------------------------ fused MLP tower (a7, §8f)
 * The whole DNNLayer (layer/interaction.py:30-46: hidden Dense(h_i, act) then
 * Dense(output_dim)) in one launch; activations stay in LDS.
 * dims[0..n_layers]: input width then each layer's units (each <= 1024);
 * W[l]: Keras kernel [dims[l], dims[l+1]]; bias[l], alpha[l] (PReLU) may be
 * NULL.  in_rows (device int32 [roundup(dims[0],16)], may be NULL): LDS
 * input column p reads Keras kernel row in_rows[p] (-1 = none), so a fused
 * producer can keep its own column order.  rs_mlp_prepared_size returns
 * floats (-1 on bad dims).                                                   */
int64_t rs_mlp_prepared_size(int n_layers, const int* dims);
int rs_mlp_prepare(int n_layers, const int* dims, const float* const* W,
                   const float* const* bias, const float* const* alpha,
                   const int32_t* in_rows, float* prepared, rs_stream_t stream);
/* head 0: y[M, dims[n_layers]] = tower(x).  head 1 (dims[n_layers] == 1):
 * y[m] = sigmoid(c0 * tower(x)[m] + c1 * extra[m]) — the DeepFM head
 * model/deepFM.py:30 (extra = FM logit, c0 = c1 = 0.5); extra may be NULL.
 * acts[l]: rs_act per layer (hidden: the DNNLayer activation; last: NONE).  */
int rs_mlp_fwd(const float* x, int64_t x_stride, int n_layers, const int* dims,
               const int* acts, const float* prepared, float* y,
               int64_t y_stride, int head, const float* extra, float c0,
               float c1, int64_t batch, rs_stream_t stream);
/* ... with an inference BatchNormalization on the input folded into the
 * tile staging: column c enters the tower as x[m, c] * in_scale[c] +
 * in_shift[c] (rs_affine_act's arithmetic; DIN.call's bn_layer before the
 * DNN, model/din.py:89), so the normalised concat never reaches HBM.        */
int rs_mlp_affine_fwd(const float* x, int64_t x_stride, const float* in_scale,
                      const float* in_shift, int n_layers, const int* dims,
                      const int* acts, const float* prepared, float* y,
                      int64_t y_stride, int head, const float* extra, float c0,
                      float c1, int64_t batch, rs_stream_t stream);
/* ... and some input columns read straight from their sources instead of x:
 * the concat pieces of rs_concat_pieces (widths / kinds / srcs / strides /
 * tables / vocabs as there; in_cols = the input column of each piece's first
 * column), e.g. DIN.call's other sparse embeddings and dense features
 * (model/din.py:64-69,84-85) beside the pooled attention — the concat is
 * never written and needs no launch of its own.  x (rows x_stride apart)
 * provides every other column (NULL if the pieces cover them all).  At most
 * 64 input columns; an out-of-range id reads a zero row and sets err_flag. */
int rs_mlp_affine_pieces_fwd(const float* x, int64_t x_stride,
                             const float* in_scale, const float* in_shift,
                             int n_layers, const int* dims, const int* acts,
                             const float* prepared, float* y, int64_t y_stride,
                             int head, const float* extra, float c0, float c1,
                             int64_t batch, int n_pieces, const int* widths,
                             const int* in_cols, const int* kinds,
                             const void* const* srcs,
                             const int64_t* src_strides,
                             const float* const* tables, const int64_t* vocabs,
                             int* err_flag, rs_stream_t stream);

/* --------------------------------------------- fused DeepFM forward (a8)
 * DeepFM.call (model/deepFM.py:23-31) in ONE launch: ids -> rows -> x (kept
 * in LDS) -> FM logit and the DNN tower -> out[b] = sigmoid(c0*dnn + c1*fm)
 * (reference: c0 = c1 = 0.5).  Arguments as rs_embed_fm_fwd plus the tower
 * (rs_mlp_*).  mlp_prepared must be packed with in_rows mapping the LDS
 * column order [emb F*k | dense nd] to Keras rows: p < F*k -> nd + p,
 * F*k <= p < F*k+nd -> p - F*k, else -1.  fm_logit (optional) receives the
 * FM logit.  rs_deepfm_fused_ok: 1 when the shape is supported (k 8 or 16,
 * kfm <= 15, 1..128 fields, tower output 1, dims[0] = nd + F*k).            */
int rs_deepfm_fused_ok(int nd, int n_fields, int k, int kfm, int n_layers,
                       const int* dims);
int rs_deepfm_fwd(const void* ids, int id_kind, int64_t id_stride,
                  const float* dense, int64_t dense_stride, int nd,
                  const float* table, const int64_t* field_offsets,
                  const int64_t* field_vocab, int n_fields, int k,
                  const float* fm_prepared, const float* w0, int kfm,
                  int n_layers, const int* dims, const int* acts,
                  const float* mlp_prepared, float c0, float c1, float* out,
                  float* fm_logit, int64_t batch, int* err_flag,
                  rs_stream_t stream);
/* rs_deepfm_fwd with the field metadata also on the host (kernel arguments
 * for n_fields <= 32, as rs_embed_fm_fwd_hm; the host arrays must equal the
 * device ones).                                                             */
int rs_deepfm_fwd_hm(const void* ids, int id_kind, int64_t id_stride,
                     const float* dense, int64_t dense_stride, int nd,
                     const float* table, const int64_t* field_offsets,
                     const int64_t* field_vocab,
                     const int64_t* field_offsets_host,
                     const int64_t* field_vocab_host, int n_fields, int k,
                     const float* fm_prepared, const float* w0, int kfm,
                     int n_layers, const int* dims, const int* acts,
                     const float* mlp_prepared, float c0, float c1, float* out,
                     float* fm_logit, int64_t batch, int* err_flag,
                     rs_stream_t stream);

/* Dense + PReLU whose alpha is [alpha_rows, N], row m using alpha row
 * m % alpha_rows: Keras Dense(N, activation=PReLU()) on a 3-D input
 * [B, alpha_rows, K] flattened to [B*alpha_rows, K] (PReLU's alpha has shape
 * input_shape[1:] = (T, N)).                                                */
int rs_dense_prelu_rows_fwd(const float* x, int64_t x_stride, const float* W,
                            const float* bias, const float* alpha,
                            int alpha_rows, float* y, int64_t y_stride,
                            int64_t M, int K, int N, rs_stream_t stream);

/* Per-column affine + activation, in place allowed: y = act(x*scale + shift).
 * Used for BatchNormalization at inference (model/din.py:89).               */
int rs_affine_act(const float* x, int64_t x_stride, const float* scale,
                  const float* shift, const float* alpha, int act, float* y,
                  int64_t y_stride, int64_t M, int N, rs_stream_t stream);

/* Dice at inference on a 2-D input (layer/interaction.py:410-425), per column
 * n: xhat = (x-mean[n])/sqrt(var[n]+eps), p = sigmoid(xhat),
 *    y = alpha[n]*(1-p)*x + p*x.  Used for DIN's dnn_activation='dice'.     */
int rs_dice_fwd(const float* x, int64_t x_stride, const float* mean,
                const float* var, float eps, const float* alpha, float* y,
                int64_t y_stride, int64_t M, int N, rs_stream_t stream);

/* Model heads: out[b] = sigmoid(c0*a[b] + c1*b[b]) (b may be NULL).
 * DeepFM: sigmoid(0.5*(fm+dnn)) (model/deepFM.py:30).                       */
int rs_sigmoid_combine(const float* a, const float* b, float c0, float c1,
                       float* out, int64_t n, rs_stream_t stream);

/* ------------------------- other interactions on the gather (§8(f) rank 3)
 * rs_embed_pair_pool_fwd: per sample, the F field rows e_c (one concatenated
 *  table, per-field offsets) pooled over the P = F(F-1)/2 pair products
 *  e_i*e_j (per dim): mode 0 = sum = 0.5((sum e)^2 - sum e^2) — NFM's
 *  bi-interaction (model/nfm.py:28) and AFM 'att' (AttentionLayer's softmax
 *  over a size-1 axis is 1, layer/interaction.py:313-318); mode 1 = mean
 *  (AFM 'avg'); mode 2 = max (AFM 'max', F <= 64).  Outputs (any subset):
 *  out[b*out_stride + out_col + j] = pooled_j and out[b*out_stride + i] =
 *  dense[b, i] for i < nd (NFM's concat([dense, emb]), model/nfm.py:29);
 *  head_out[b] = sigmoid^n_sigmoid(pooled @ head_w + head_b) (AFMLayer's
 *  Dense(1) + sigmoid, then AFM.call's second sigmoid: n_sigmoid = 2).
 * rs_pair_products_fwd: InteractionLayer (layer/interaction.py:280-297):
 *  e [batch, F*k] (row stride e_stride) -> out [batch, P, k], pairs i<j
 *  row-major.
 * rs_ffm_fwd: FFMLayer.call + FFM.call (layer/interaction.py:134-163,
 *  model/ffm.py:20-22) on label-encoded ids: x = [dense | one-hot], feature
 *  f = nd + field_offsets[c] + id; v [feature_num, (nd+F)*k], w
 *  [feature_num]; out[b] = sigmoid^n_sigmoid(w0 + x@w + sum_{f<g}
 *  <field_f, field_g>), field = x @ v; k divides 64, (nd+F)*k <= 1024.      */
int rs_embed_pair_pool_fwd(const void* ids, int id_kind, int64_t id_stride,
                           const float* table, const int64_t* field_offsets,
                           const int64_t* field_vocab, int n_fields, int k,
                           int mode, const float* dense, int64_t dense_stride,
                           int nd, float* out, int64_t out_stride, int out_col,
                           const float* head_w, const float* head_b,
                           int n_sigmoid, float* head_out, int64_t batch,
                           int* err_flag, rs_stream_t stream);
int rs_pair_products_fwd(const float* e, int64_t e_stride, int n_fields, int k,
                         int64_t batch, float* out, rs_stream_t stream);
/* AttentionLayer.call (layer/interaction.py:310-319) on x [batch, n_rows, k]
 * (row stride x_stride): its softmax runs over a size-1 axis (every score is
 * exactly 1), so out[b, j] = sum_p x[b, p, j].                             */
int rs_attention_pool_fwd(const float* x, int64_t x_stride, int n_rows, int k,
                          int64_t batch, float* out, rs_stream_t stream);
int rs_ffm_fwd(const void* ids, int id_kind, int64_t id_stride,
               const float* dense, int64_t dense_stride, int nd,
               const float* v, const float* w, const float* w0,
               const int64_t* field_offsets, const int64_t* field_vocab,
               int n_fields, int k, int n_sigmoid, float* out, int64_t batch,
               int* err_flag, rs_stream_t stream);

/* ------------------------------------------ training (§8(f) rank 4)
 * rs_fm_train_step: one SGD step of the FM model (model/fm.py:14-23 +
 * utils/compile_fit.py:9-15) on a batch in compact form — dense [B, nd] and
 * label codes ids [B, F] standing for x = [dense | one-hot] (one-hot column
 * nd + field_offsets[c] + id, utils/dataset.py:47-48) — with the FMLayer
 * weights w0 (1), w1 (n_rows), v (n_rows, k) updated in place:
 *   y = w0 + x@w1 + 0.5 sum_f [(x@v)_f^2 - (x^2@v^2)_f],
 *   dL/dy_b = (sigmoid(y_b) - labels_b) / B   (Keras binary_crossentropy on
 *   the sigmoid's logits, batch mean), l2 regularisers l2_w on w1 and l2_v
 *   on v (FMLayer.build, layer/interaction.py:97-104), SGD with rate lr.
 * Every row decays (the regulariser's dense gradient); the looked-up rows
 * get their summed gradient through a deterministic sort + segmented sum.
 * loss (optional, [B]): per-sample cross-entropy before the step.
 * workspace: rs_fm_train_workspace_size(B, F, k, nd) bytes (device).       */
int64_t rs_fm_train_workspace_size(int64_t batch, int n_fields, int k, int nd);
int rs_fm_train_step(const void* ids, int id_kind, int64_t id_stride,
                     const float* dense, int64_t dense_stride, int nd,
                     const int64_t* field_offsets, const int64_t* field_vocab,
                     int n_fields, int k, float* w0, float* w1, float* v,
                     int64_t n_rows, const float* labels, int64_t batch,
                     float lr, float l2_w, float l2_v, void* workspace,
                     float* loss, int* err_flag, rs_stream_t stream);

/* rs_dropout: DNNLayer's Dropout(rate) in training (layer/interaction.py:35,44;
 * active under compile_fit's model.fit, utils/compile_fit.py:14), in place on
 * x[rows, cols] (row stride ld): x <- keep ? x / (1 - rate) : 0 with
 * keep = u >= rate, u from Philox4x32-10 (key = seed, counter =
 * (offset + row*cols + col) / 4, word (offset + e) % 4, u = (word >> 8) 2^-24).
 * offset % 4 == 0; callers advance it by 4*ceil(rows*cols/4) per draw.  The
 * same (seed, offset) applied to dL/dx is the backward (the mask is never
 * stored).  TF's own draws cannot be reproduced; oracle.dropout_multiplier
 * restates this generator exactly.                                          */
int rs_dropout(float* x, int64_t ld, int64_t rows, int64_t cols, float rate,
               uint64_t seed, uint64_t offset, rs_stream_t stream);
/* rs_dropout_at: the same draw at offset *base + offset, with the base read
 * on the device (a per-generator counter in device memory), so a captured
 * hipGraph replays fresh masks; rs_dropout_advance adds inc (a multiple of 4)
 * to *base on the stream — the training steps call it once, after the
 * backward's redraws, with the step's total.                                */
int rs_dropout_at(float* x, int64_t ld, int64_t rows, int64_t cols, float rate,
                  uint64_t seed, const uint64_t* base, uint64_t offset,
                  rs_stream_t stream);
int rs_dropout_advance(uint64_t* base, uint64_t inc, rs_stream_t stream);

/* DeepFM training (model/deepFM.py + utils/compile_fit.py; the host layer
 * DeepFM.train_step composes these with rs_embed_gather / rs_dense_fwd /
 * rs_fm_fwd):
 * rs_gemm: C[M,N] = alpha op(A)[M,K] op(B)[K,N] + beta C (row-major; op =
 *  transpose when trans_*), then C *= (mask > 0) if mask (ReLU backward);
 *  deterministic (each output's K sum in one fixed order).  With a
 *  workspace of rs_gemm_workspace_size(M, N, K) bytes (0 = not needed) a
 *  launch of few output tiles splits K into slices summed in slice order.
 * rs_col_sum: out[n] = sum_m A[m,n] (bias gradients), fixed-order trees.
 * rs_sgd_update: w -= lr (grad + 2 l2 w) (Keras SGD + l2 regulariser).
 * rs_head_grad: z = c_fm fm + c_dnn dnn (DeepFM: 0.5, 0.5),
 *  g = (sigmoid(z) - t)/B -> g_fm = c_fm g, g_dnn = c_dnn g, loss (optional).
 * rs_fm_x_grad: dx[b,i] += g_b (w1_i + sum_f v_if s_bf - x_bi sum_f v_if^2)
 *  (FMLayer w.r.t. its input; s = x @ v).
 * rs_fm_param_grads: dw1 = x^T g, dv = x^T (g s) - (x^2)^T g * v, dw0 =
 *  sum g (no l2 terms; kfm <= 32).
 * rs_embedding_sgd: table[off_c + id(b,c)] -= lr * grad[b, c*k : c*k+k]
 *  summed over duplicate rows in lookup order (stable sort + segmented sum:
 *  Keras' IndexedSlices scatter-add); workspace:
 *  rs_embedding_sgd_workspace_size(batch * n_fields) bytes.                 */
/* rs_sort_pairs_u32: stable ascending sort of (key, val) pairs by the low
 *  `bits` bits of key (LSD radix, 8 bits a pass; equal keys keep their input
 *  order), the grouping step of every row-sparse scatter-add here
 *  (rs_embedding_sgd, rs_fm_train_step, rs_shard_dedup_route beyond 4096
 *  samples) — Keras' IndexedSlices accumulation groups the same rows
 *  (utils/compile_fit.py:9-15 via SGD on the Embedding); in != out,
 *  workspace: rs_sort_pairs_workspace_size(n) bytes.
 * rs_inclusive_sum_i32: out[i] = in[0] + ... + in[i] (in == out allowed),
 *  workspace: rs_inclusive_sum_workspace_size(n) bytes.                    */
int64_t rs_sort_pairs_workspace_size(int64_t n);
int rs_sort_pairs_u32(const uint32_t* key_in, const uint32_t* val_in,
                      uint32_t* key_out, uint32_t* val_out, int64_t n,
                      int bits, void* workspace, rs_stream_t stream);
int64_t rs_inclusive_sum_workspace_size(int64_t n);
int rs_inclusive_sum_i32(const int32_t* in, int32_t* out, int64_t n,
                         void* workspace, rs_stream_t stream);
int64_t rs_gemm_workspace_size(int64_t M, int64_t N, int64_t K);
int rs_gemm(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
            float alpha, const float* A, int64_t lda, const float* B,
            int64_t ldb, float beta, float* C, int64_t ldc, const float* mask,
            int64_t ldm, void* workspace, int64_t workspace_bytes,
            rs_stream_t stream);
int rs_col_sum(const float* A, int64_t lda, int64_t M, int64_t N, float* out,
               rs_stream_t stream);
/* rs_col_sum over many rows: slices of 256 rows (fewer, down to 16, when
 * that leaves < 64 slices) summed into a workspace of
 * rs_col_sum_workspace_size(M, N) bytes, then the slices in order
 * (deterministic); without room (or one slice) it is rs_col_sum.           */
int64_t rs_col_sum_workspace_size(int64_t M, int64_t N);
int rs_col_sum_split(const float* A, int64_t lda, int64_t M, int64_t N,
                     float* out, void* workspace, int64_t workspace_bytes,
                     rs_stream_t stream);
int rs_sgd_update(float* w, const float* grad, int64_t n, float lr, float l2,
                  rs_stream_t stream);
/* rs_sgd_update over `count` tensors (host arrays of device pointers, sizes
 * and per-tensor l2) in one launch per 32 tensors: the optimizer step of a
 * model's dense parameters (Keras' SGD.apply_gradients over the variable
 * list, utils/compile_fit.py:11 / model/pnn.py:81), same arithmetic.       */
int rs_sgd_update_multi(int count, float* const* w, const float* const* grad,
                        const int64_t* n, const float* l2, float lr,
                        rs_stream_t stream);
int rs_head_grad(const float* fm, const float* dnn, const float* labels,
                 int64_t batch, float c_fm, float c_dnn, float* g_fm,
                 float* g_dnn, float* loss, rs_stream_t stream);
/* PNN training (the reference's GradientTape loop, model/pnn.py:74-85):
 * rs_bce_prob_grad: tf.reduce_mean(losses.binary_crossentropy(y[B],
 *  pre[B,1])) on the DNN LOGIT as Keras computes it — pre clipped to
 *  [1e-7, 1-1e-7], labels broadcast against the [B,1] output (per sample i
 *  the mean over j of BCE(y_j, pre_i)): loss[i] = -(ybar log(q_i+eps) +
 *  (1-ybar) log(1-q_i+eps)), g[i] = dL/dpre_i (0 outside the clip range).
 * rs_inner_product_bwd: InnerProductLayer backward (layer/interaction.py:
 *  170-183): demb[b,i,:] = dflat[b,i,:] + sum_{j!=i} dinner[b,p(i,j)]
 *  emb[b,j,:] (p = the row-major pair index); 2 <= n_fields <= 64, k <= 64. */
int rs_bce_prob_grad(const float* pred, int64_t pred_stride,
                     const float* labels, int64_t batch, float* g, float* loss,
                     rs_stream_t stream);
int rs_inner_product_bwd(const float* emb, int64_t emb_stride,
                         const float* dinner, int64_t dinner_stride,
                         const float* dflat, int64_t dflat_stride, int n_fields,
                         int k, int64_t batch, float* demb, int64_t demb_stride,
                         rs_stream_t stream);
/* NFM Bi-Interaction backward (model/nfm.py:28, 3-D embeddings; NFM
 * training): demb[b, f*k + c] = dbi[b, c] (S_bc - e_bfc), S = sum_f e_f.      */
int rs_bi_interaction_bwd(const float* emb, int64_t emb_stride,
                          const float* dbi, int64_t dbi_stride, int n_fields,
                          int k, int64_t batch, float* demb,
                          int64_t demb_stride, rs_stream_t stream);
/* OuterProductLayer backward (layer/interaction.py:200-215, PNN modes
 * 'outer' / 'both'): o_p = e_j^T W_p e_i, W_p[a][c] = W[a,p,c], W [k, P, k].
 * rs_outer_product_bwd ADDS to demb[b, f*k ..]: sum_{j>f} g_p e_j W_p +
 *  sum_{i<f} g_p e_i W_p^T (g = dout[b, p], pairs in order).
 * rs_outer_product_w_grad: dW[a,p,c] = sum_b g_bp e_j[b,a] e_i[b,c].
 * 2 <= n_fields <= 64, 1 <= k <= 16; fp32 MFMA, deterministic.              */
int rs_outer_product_bwd(const float* emb, int64_t emb_stride,
                         const float* dout, int64_t dout_stride, const float* W,
                         int n_fields, int k, int64_t batch, float* demb,
                         int64_t demb_stride, rs_stream_t stream);
int rs_outer_product_w_grad(const float* emb, int64_t emb_stride,
                            const float* dout, int64_t dout_stride,
                            int n_fields, int k, int64_t batch, float* dW,
                            rs_stream_t stream);
/* DIN training (compile_fit on model/din.py:56-95, training=True; the host
 * layer DIN.train_step composes these with rs_dense_fwd / rs_gemm /
 * rs_col_sum / rs_sgd_update / rs_embedding_sgd):
 * rs_din_att_concat: out[b*T+t] = [q_b, s_bt, q_b - s_bt, q_b * s_bt]
 *  (the attention unit input, layer/interaction.py:381-391); item [B,K],
 *  seq [B*T,K], out [B*T,4K] dense rows.
 * rs_din_att_concat_bwd: from d = dL/dout: dq[b] += sum_t (d0 + d2 + s d3)
 *  (row stride dq_stride), dseq[b*T+t] += d1 - d2 + q d3.
 * rs_prelu_rows_fwd / _bwd: Keras PReLU on rows, y = max(z,0) +
 *  alpha[(r mod period), c] min(z,0) (the attention's [T,h] alphas: period
 *  T; a Dense layer's [N]: period 1); bwd writes dz = dy (z>0 ? 1 : alpha)
 *  and dalpha[p,c] = sum_{r = p mod period} dy min(z,0) (the split column
 *  sums below; M a multiple of period); workspace:
 *  rs_prelu_rows_bwd_workspace_size(M, N, period) bytes.
 * rs_masked_softmax_pool: s = score, or -2^32+1 where hist[b,0..T) == 0
 *  (the first behaviour feature, model/din.py:80); a = softmax_T(s) [B,T];
 *  out[b] = sum_t a_t seq[b*T+t] (:396-404).  T <= 512.
 * rs_masked_softmax_pool_bwd: from datt: ds[b,t] = live ? a_t (da_t -
 *  sum_s a_s da_s) : 0 with da_t = datt . seq_t; dseq[b*T+t] = a_t datt
 *  (stored, not accumulated).
 * rs_bn_train_fwd: BatchNormalization in training mode — per column the
 *  batch mean and biased variance into mean / var, y = (x - mean)
 *  rsqrt(var + eps) gamma + beta, and (when non-NULL) moving = momentum
 *  moving + (1 - momentum) batch stat.
 * rs_bn_train_bwd: dgamma = sum dy xhat, dbeta = sum dy, dx = gamma
 *  rsqrt(var+eps) (dy - dbeta/B - xhat dgamma/B).                          */
int rs_din_att_concat(const float* item, const float* seq, int64_t batch,
                      int T, int K, float* out, rs_stream_t stream);
int rs_din_att_concat_bwd(const float* d, const float* item, const float* seq,
                          int64_t batch, int T, int K, float* dq,
                          int64_t dq_stride, float* dseq, rs_stream_t stream);
int rs_prelu_rows_fwd(const float* z, int64_t M, int N, const float* alpha,
                      int period, float* y, rs_stream_t stream);
int64_t rs_prelu_rows_bwd_workspace_size(int64_t M, int N, int period);
int rs_prelu_rows_bwd(const float* z, const float* dy, int64_t M, int N,
                      const float* alpha, int period, float* dz,
                      float* dalpha, void* workspace, int64_t workspace_bytes,
                      rs_stream_t stream);
/* rs_din_att_prelu_bwd: the whole backward of the PReLU attention unit
 * with two hidden layers (layer/interaction.py:366-395; default (80, 40)) in
 * one launch + a fixed-order partial sum: from h0 [B*T, K0] (the concat
 * [q, k, q-k, q*k]), the pre-activations z1 [B*T, h1], z2 [B*T, h2], ds
 * [B*T] (dL/dscore), the kernels W1 [K0, h1], W2 [h1, h2], the PReLU alphas
 * [T, h1] / [T, h2] and the score kernel wo [h2], writes dh0 [B*T, K0] and
 * dW1, db1, dalpha1, dW2, db2, dalpha2, dwo [h2], dbo [1].  Shapes with T,
 * K0, h1, h2 <= 128, multiples of 4, whose sample fits in LDS:
 * rs_din_att_prelu_bwd_workspace_size returns -1 for the others.           */
/* rs_din_att_prelu_fwd: the unit's forward under fit for the same shapes:
 * z1 = h0 W1 + b1, z2 = prelu(z1; alpha1) W2 + b2 (kept for the backward),
 * score = prelu(z2; alpha2) wo + bo [B*T], one launch.                      */
int rs_din_att_prelu_fwd(const float* h0, const float* W1, const float* b1,
                         const float* alpha1, const float* W2,
                         const float* b2, const float* alpha2,
                         const float* wo, const float* bo, int64_t batch,
                         int T, int K0, int h1, int h2, float* z1, float* z2,
                         float* score, rs_stream_t stream);
int64_t rs_din_att_prelu_bwd_workspace_size(int64_t batch, int T, int K0,
                                            int h1, int h2);
int rs_din_att_prelu_bwd(const float* h0, const float* z1, const float* z2,
                         const float* ds, const float* W1, const float* W2,
                         const float* alpha1, const float* alpha2,
                         const float* wo, int64_t batch, int T, int K0, int h1,
                         int h2, float* dh0, float* dW1, float* db1,
                         float* dalpha1, float* dW2, float* db2,
                         float* dalpha2, float* dwo, float* dbo,
                         void* workspace, int64_t workspace_bytes,
                         rs_stream_t stream);
int rs_masked_softmax_pool(const float* score, const void* hist,
                           int hist_kind, int64_t hist_stride,
                           const float* seq, int64_t batch, int T, int K,
                           float* a, float* out, int64_t out_stride,
                           rs_stream_t stream);
int rs_masked_softmax_pool_bwd(const float* a, const void* hist,
                               int hist_kind, int64_t hist_stride,
                               const float* seq, const float* datt,
                               int64_t datt_stride, int64_t batch, int T,
                               int K, float* ds, float* dseq,
                               rs_stream_t stream);
int rs_bn_train_fwd(const float* x, int64_t x_stride, int64_t batch, int D,
                    const float* gamma, const float* beta, float eps,
                    float momentum, float* moving_mean, float* moving_var,
                    float* mean, float* var, float* y, int64_t y_stride,
                    rs_stream_t stream);
int rs_bn_train_bwd(const float* x, int64_t x_stride, int64_t batch, int D,
                    const float* mean, const float* var, const float* gamma,
                    float eps, const float* dy, int64_t dy_stride, float* dx,
                    int64_t dx_stride, float* dgamma, float* dbeta,
                    rs_stream_t stream);
/* Dice in training (layer/interaction.py:416-425 under fit, DIN with
 * att_attention / dnn_activation 'dice'), x [M, N] dense rows (the
 * attention's [B, T, 4k] as [B*T, 4k]): its BatchNormalization(center=False,
 * scale=False) with the batch's per-column mean and biased variance (into
 * mean / var, moving averages moved with momentum when non-NULL);
 * y = alpha (1 - p) x + p x, p = sigmoid((x - mean) rsqrt(var + eps)).
 * rs_dice_train_bwd: dx = dy (alpha (1-p) + p) + the batch-norm backward of
 * dL/dxhat = dy (1 - alpha) x p (1 - p); dalpha = sum dy (1 - p) x.
 * Workspace: rs_dice_train_workspace_size(M, N) bytes.  Deterministic.     */
int64_t rs_dice_train_workspace_size(int64_t M, int N);
int rs_dice_train_fwd(const float* x, int64_t M, int N, const float* alpha,
                      float eps, float momentum, float* moving_mean,
                      float* moving_var, float* mean, float* var, float* y,
                      void* workspace, int64_t workspace_bytes,
                      rs_stream_t stream);
int rs_dice_train_bwd(const float* x, int64_t M, int N, const float* alpha,
                      const float* mean, const float* var, float eps,
                      const float* dy, float* dx, float* dalpha,
                      void* workspace, int64_t workspace_bytes,
                      rs_stream_t stream);
/* rs_head_grad with g = scale (sigmoid(z) - t) (scale > 0): the sharded
 * DeepFM step's local batch is a 1/world share of the global batch mean,
 * scale = 1 / (world * batch).                                             */
int rs_head_grad_scaled(const float* fm, const float* dnn, const float* labels,
                        int64_t batch, float c_fm, float c_dnn, float scale,
                        float* g_fm, float* g_dnn, float* loss,
                        rs_stream_t stream);
int rs_fm_x_grad(const float* x, int64_t ldx, const float* s, const float* w1,
                 const float* v, int64_t batch, int d, int kfm, const float* g,
                 float* dx, int64_t lddx, rs_stream_t stream);
int rs_fm_param_grads(const float* x, int64_t ldx, const float* s,
                      const float* v, int64_t batch, int d, int kfm,
                      const float* g, float* dw1, float* dv, float* dw0,
                      rs_stream_t stream);
/* rs_fm_param_grads with s rows lds floats apart and g ldg floats apart
 * (the sharded backward's interleaved [s | g] records); dw0 NULL = skip.   */
int rs_fm_param_grads_strided(const float* x, int64_t ldx, const float* s,
                              int64_t lds, const float* g, int64_t ldg,
                              const float* v, int64_t batch, int d, int kfm,
                              float* dw1, float* dv, float* dw0,
                              rs_stream_t stream);
/* CrossNet training (layer/interaction.py:75-83, DCN.train_step):
 * rs_cross_train_fwd: x_{l+1} = x0 (x_l . w_l) + b_l + x_l for l < L;
 *  W, b [L, d] (row l = w_l, b_l); keeps xs [L, B, d] (x_1 .. x_L) and
 *  g [L, B] (g_l = x_l . w_l); x_L also to xl_out (row stride ldo; may be
 *  NULL).  d <= 2048.
 * rs_cross_train_bwd: from dxl = dL/dx_L: deltas [L, B, d] (delta_{l+1} for
 *  db_l = sum_b delta_{l+1}), s [L, B] (s_l = x0 . delta_{l+1}, for dw_l =
 *  sum_b s_l x_l), and dx += delta_0 + sum_l g_l delta_{l+1} (dL/dx0).      */
int rs_cross_train_fwd(const float* x0, int64_t ldx, int d, int n_layers,
                       const float* W, const float* b, int64_t batch,
                       float* xs, float* g, float* xl_out, int64_t ldo,
                       rs_stream_t stream);
int rs_cross_train_bwd(const float* x0, int64_t ldx, int d, int n_layers,
                       const float* W, int64_t batch, const float* g,
                       const float* dxl, int64_t lddxl, float* deltas,
                       float* s, float* dx, int64_t lddx,
                       rs_stream_t stream);
/* rs_embedding_sgd with the gradient row of lookup (b, c) at grad[b *
 * grad_stride + c * grad_field_stride] (k for one row per lookup; 0 for one
 * row per sample shared by all its fields — the FFM step).                 */
int rs_embedding_sgd_strided(float* table, int64_t n_rows, int k,
                             const void* ids, int id_kind, int64_t id_stride,
                             const int64_t* field_offsets,
                             const int64_t* field_vocab, int n_fields,
                             int64_t batch, const float* grad,
                             int64_t grad_stride, int64_t grad_field_stride,
                             float lr, void* workspace, int* err_flag,
                             rs_stream_t stream);
/* FFM training (compile_fit on FFM, model/ffm.py:20-22; FFM.train_step
 * composes it with rs_gemm / rs_col_sum / rs_sgd_update / rs_l2_decay /
 * rs_embedding_sgd_strided): rs_ffm_train_fwd computes, per sample, Fm[f,c]
 * = sum_i x_i v[i,f,c] (v [feature_num, nd+F, k]; the nd dense rows and row
 * nd + field_offsets[c] + id of each field, an out-of-range id being
 * tf.one_hot's zero row), z = w0 + x.w + 0.5(|sum_f Fm_f|^2 - sum_f |Fm_f|^2),
 * g[b] = (sigmoid(z) - t)/B, loss[b] (optional) and G[b, f*k + c] =
 * g (T_c - Fm[f,c]), T = sum_f Fm_f.  (nd + F) * k <= 4096, k <= 64.
 * rs_l2_decay: w -= lr * 2 l2 w over n floats (Keras l2 on every row).      */
int rs_ffm_train_fwd(const void* ids, int id_kind, int64_t id_stride,
                     const float* dense, int64_t dense_stride, int nd,
                     const float* v, const float* w, const float* w0,
                     const int64_t* field_offsets, const int64_t* field_vocab,
                     int n_fields, int k, const float* labels, int64_t batch,
                     float* G, float* g, float* loss, rs_stream_t stream);
int rs_l2_decay(float* w, int64_t n, float lr, float l2, rs_stream_t stream);
int64_t rs_embedding_sgd_workspace_size(int64_t n_lookups);
int rs_embedding_sgd(float* table, int64_t n_rows, int k, const void* ids,
                     int id_kind, int64_t id_stride,
                     const int64_t* field_offsets, const int64_t* field_vocab,
                     int n_fields, int64_t batch, const float* grad,
                     int64_t grad_stride, float lr, void* workspace,
                     int* err_flag, rs_stream_t stream);

/* -------------------------------------- row-sharded lookup (§8(e), cfg 5)
 * Global row of (b,c) = field_offsets[c] + id(b,c).  Rows are split across
 * `world` ranks in blocks of `rows_per_rank` (owner = row / rows_per_rank).
 *  rs_shard_bucketize: counts[r] = #lookups owned by rank r; perm[i] = the
 *   position of lookup i (= b*F + c) in owner-major order; send_rows[perm[i]]
 *   = local row index on the owner.  Stable within each owner.
 *   workspace: rs_shard_workspace_size(batch*n_fields, world) bytes, device,
 *   zero-filled once when allocated (its tail holds the control words of the
 *   one-pass slotted kernel, which leaves them ready for the next call); one
 *   workspace per stream — concurrent calls must not share it.
 *  rs_gather_rows: out[i] = table[rows[i]] (k floats), local shard.
 *  rs_unpermute_rows: dst[i] = src[perm[i]] (k floats per row).            */
int64_t rs_shard_workspace_size(int64_t n_lookups, int world);
int rs_shard_bucketize(const void* ids, int id_kind, int64_t id_stride,
                       const int64_t* field_offsets, const int64_t* field_vocab,
                       int n_fields, int64_t batch, int64_t rows_per_rank,
                       int world, int32_t* counts, int32_t* perm,
                       int32_t* send_rows, void* workspace, int* err_flag,
                       rs_stream_t stream);

/* Fixed-capacity ("slotted") variant for a host-sync-free exchange: every
 * (rank -> owner) message is exactly `cap` slots, so both all-to-alls have
 * equal, host-known splits.  send_slots [world*cap]: slots not used by this
 * step keep their previous content (fill the buffer with -1 once, when it is
 * allocated: -1 is served as a zero row, a stale slot as a valid row of the
 * owner's shard that no lookup reads); slot_of [B*F]: the slot of lookup
 * b*F+c, or -1 when its owner's slots overflowed (*overflow_flag set; redo the
 * step with the exact protocol) or its id is out of range (*err_flag set).
 * The returned rows are then addressed by slot_of as int32 ids of a single
 * [world*cap, k] table: rs_embed_fm_fwd(ids = slot_of, offsets 0, vocab
 * world*cap) computes the FM straight from the exchange buffer.
 * One launch: stable per-owner ranks in LDS + a decoupled look-back over the
 * preceding blocks' per-owner totals (single-pass chained scan).            */
int rs_shard_slot_bucketize(const void* ids, int id_kind, int64_t id_stride,
                            const int64_t* field_offsets,
                            const int64_t* field_vocab, int n_fields,
                            int64_t batch, int64_t rows_per_rank, int world,
                            int cap, int32_t* counts, int32_t* slot_of,
                            int32_t* send_slots, void* workspace, int* err_flag,
                            int* overflow_flag, rs_stream_t stream);
int rs_gather_rows(const float* table, int64_t n_rows, int k,
                   const int32_t* rows, int64_t n, float* out, int* err_flag,
                   rs_stream_t stream);
int rs_unpermute_rows(const float* src, const int32_t* perm, int k, int64_t n,
                      float* dst, rs_stream_t stream);

/* ------------------- row-sharded FM, partial protocol (§8(e), default)
 * A block split of the concatenated table gives every owner o a contiguous
 * FIELD range [field_lo(o), field_lo(o) + n_owned(o)).  Instead of returning
 * 64-B rows, the owner returns per-sample FM partials over the fields it
 * holds (the FM's first stage x@[v|w1] and x^2@|v|^2 is linear in the rows),
 * and the requester finishes the FM (FMLayer.call, layer/interaction.py:
 * 106-114; EmbedLayer.call, layer/core.py:273-280, for the lookup):
 *  rs_fm_partial_width(kfm): floats per partial record, P = roundup(kfm+2, 4):
 *   [s_0 .. s_{kfm-1}, x@w1, sum_i x_i^2 |v_i|^2, 0-pad].
 *  rs_shard_field_route: owner_fields [world][2] int32 = (field_lo, n_owned)
 *   per owner; send = world*batch records of rec_stride int32 words (owner-
 *   major), word j < slot_stride (slot_stride >= every n_owned) of record
 *   (o, b) = local row of lookup (b, field_lo(o)+j) when o owns it, else -1.
 *   Those words are all written; words >= slot_stride are left untouched;
 *   out-of-range id -> *err_flag.
 *  rs_shard_owner_fm: local_rows = n_pairs records of rec_stride words (the
 *   received messages, requester-major), the owner's shard [shard_rows, k]
 *   and the packed FM image of the WHOLE model (rs_fm_prepare with nd,
 *   n_fields) -> partial records (P floats, partial_stride floats apart) over
 *   fields field_lo .. field_lo+n_owned-1 (-1 rows contribute 0; a local row
 *   >= shard_rows sets *err_flag).
 *  rs_shard_fm_combine: partial records [world][batch] (partial_stride floats
 *   apart, one block per owner) + dense [batch, nd] -> logit[batch]; owners
 *   summed in rank order.
 *  A pipelined exchange interleaves both messages in ONE buffer: record
 *   (peer, b) = [slot_stride row ids of batch t | P partial floats of batch
 *   t-1], rec_stride = partial_stride = slot_stride + P, partials at +slot_stride
 *   words: one all-to-all per batch (sharded.py forward_stream).            */
int rs_fm_partial_width(int kfm);
int rs_shard_field_route(const void* ids, int id_kind, int64_t id_stride,
                         const int64_t* field_offsets,
                         const int64_t* field_vocab, int n_fields,
                         int64_t batch, int64_t rows_per_rank, int world,
                         const int32_t* owner_fields, int slot_stride,
                         int64_t rec_stride, int32_t* send, int* err_flag,
                         rs_stream_t stream);
/* Row protocol on the same field-range records (ShardedDeepFM, config 5: the
 * DNN needs every row at the requester, so rows come back instead of FM
 * partials; EmbedLayer.call, layer/core.py:273-280, sharded):
 *  rs_shard_row_route: rs_shard_field_route with rec_stride = slot_stride,
 *   plus slot_of[b*n_fields + c] = the record word (o*batch + b)*slot_stride
 *   + j of lookup (b, c) (o = its owner, j = c - field_lo(o)), or -1 for an
 *   out-of-range id (*err_flag set).  The owner answers the received words
 *   with rs_gather_rows (-1 -> zero row) into [world*batch*slot_stride, k];
 *   after the row all-to-all, lookup (b, c)'s row is got[slot_of[b*F + c]],
 *   so rs_deepfm_fwd(ids = slot_of, offsets 0, vocab world*batch*slot_stride,
 *   table = got) runs the whole DeepFM forward straight from the exchange
 *   buffer.  Fixed sizes, no scan, no capacity, no overflow.                 */
/* Row-id deduplication before the sharded row exchange (ShardedDeepFM with
 * dedup): the rank sends each owner only the DISTINCT rows it needs, in a
 * fixed-capacity message of `cap` words per owner (send[world*cap]: distinct
 * local row u of owner o at word o*cap + u, in row order; unused words -1,
 * served as zero rows by rs_gather_rows).  slot_of[b*n_fields + c] = o*cap +
 * u, the reply row of lookup (b, c) after the row all-to-all (rs_deepfm_fwd
 * with ids = slot_of, vocab world*cap, reads the exchange buffer unchanged);
 * -1 for a bad id (*err_flag) or a distinct row past `cap` (*overflow_flag:
 * the caller redoes the step without dedup).  For
 * batch <= 4096, n_fields <= 1024 and world <= 4096, one workgroup per
 * field dedups its lookups in an LDS hash table and numbers each owner's
 * distinct rows field by field in order of first occurrence (the
 * concatenated table's fields occupy increasing, disjoint row ranges;
 * field_offsets[c] + field_vocab[c] > field_offsets[c+1] sets
 * RS_FLAG_LAYOUT), and a second launch scatters — no sort; larger batches
 * use a device-wide radix sort and number the rows in row order.  Either
 * way the numbering is deterministic.
 * rs_shard_dedup_grad (backward, same workspace, after the route of the same
 * step): dst[slot] = sum of the gradient rows grad[b*grad_stride + c*k ..]
 * of every lookup of that distinct row, in lookup order (the lookups grouped
 * by row first — on the hash path by a per-field launch of its own — then
 * summed in fixed chunk pieces, so hot rows stay parallel) — one gradient
 * row per distinct row travels back to its owner.  Workspace: rs_shard_dedup_workspace_size(batch*n_fields,
 * world) bytes.                                                            */
int64_t rs_shard_dedup_workspace_size(int64_t n_lookups, int world);
int rs_shard_dedup_route(const void* ids, int id_kind, int64_t id_stride,
                         const int64_t* field_offsets,
                         const int64_t* field_vocab, int n_fields,
                         int64_t batch, int64_t rows_per_rank, int world,
                         int64_t cap, int32_t* send, int32_t* slot_of,
                         void* workspace, int* err_flag, int* overflow_flag,
                         rs_stream_t stream);
int rs_shard_dedup_grad(const float* grad, int64_t grad_stride, int n_fields,
                        int k, int64_t batch, int world, const int32_t* slot_of,
                        void* workspace, float* dst, rs_stream_t stream);

/* Sharded DeepFM backward (ShardedDeepFM.train_step): rs_scatter_rows
 * writes lookup j = b*n_fields + c's gradient row src[b*src_stride + c*k ..]
 * into dst[slot_of[j]] (slot_of < 0 skipped) — the row-exchange layout, so
 * the reverse all-to-all returns every owner the dL/drow of the rows it
 * served, aligned with its received row ids (rs_embedding_sgd on those ids
 * then sums duplicates in record order).                                   */
int rs_scatter_rows(const float* src, int64_t src_stride, int n_fields, int k,
                    const int32_t* slot_of, int64_t batch, float* dst,
                    rs_stream_t stream);
int rs_shard_row_route(const void* ids, int id_kind, int64_t id_stride,
                       const int64_t* field_offsets, const int64_t* field_vocab,
                       int n_fields, int64_t batch, int64_t rows_per_rank,
                       int world, const int32_t* owner_fields, int slot_stride,
                       int32_t* send, int32_t* slot_of, int* err_flag,
                       rs_stream_t stream);
int rs_shard_owner_fm(const int32_t* local_rows, int64_t rec_stride,
                      int field_lo, int n_owned, const float* shard,
                      int64_t shard_rows, int nd, int n_fields, int k,
                      const float* prepared, int kfm, float* partial,
                      int64_t partial_stride, int64_t n_pairs, int* err_flag,
                      rs_stream_t stream);
int rs_shard_fm_combine(const float* partials, int64_t partial_stride,
                        int world, int64_t batch,
                        const float* dense, int64_t dense_stride, int nd,
                        int n_fields, int k, const float* prepared,
                        const float* w0, int kfm, float* logit,
                        rs_stream_t stream);

/* Sharded FM training (sharded.py ShardedEmbeddingFM.train_step;
 * utils/compile_fit.py:9-15 on the FM logit, data parallel over the ranks):
 *  rs_shard_fm_combine_grad: rs_shard_fm_combine that also writes, per
 *   sample, the record gs[b] = [s_0 .. s_{kfm-1} | g] (gs_stride floats
 *   apart; s = x @ v over the whole sample, g = (sigmoid(logit) - label) *
 *   grad_scale, grad_scale = 1 / global batch) and the BCE loss (optional).
 *  rs_shard_owner_fm_grad: owner side of the backward.  recv = the forward's
 *   received row-id records (n_pairs of rec_stride words, requester-major),
 *   gs = every requester's [s | g] records in the same pair order (an
 *   all-gather).  For the owned fields field_lo .. +n_owned: rows_ws [n_pairs,
 *   n_owned*k] = the rows (absent -> 0); drows [n_pairs, n_owned*k] =
 *   dL/drow = g (w1_e + v_e . s - x_e |v_e|^2); dw1 [n_owned*k] and dv
 *   [n_owned*k, kfm] = this owner's part of the FM parameter gradients of
 *   those columns (fixed-order trees; summed over owners by an all-reduce).
 *   w1 / v are the WHOLE model's [d, 1] / [d, kfm].  The row update is then
 *   rs_embedding_sgd on recv (ids = local rows, -1 skipped) and drows.     */
int rs_shard_fm_combine_grad(const float* partials, int64_t partial_stride,
                             int world, int64_t batch, const float* dense,
                             int64_t dense_stride, int nd, int n_fields, int k,
                             const float* prepared, const float* w0, int kfm,
                             const float* labels, float grad_scale,
                             float* logit, float* gs, int64_t gs_stride,
                             float* loss, rs_stream_t stream);
int rs_shard_owner_fm_grad(const int32_t* recv, int64_t rec_stride,
                           int field_lo, int n_owned, const float* shard,
                           int64_t shard_rows, int nd, int k, const float* w1,
                           const float* v, int kfm, const float* gs,
                           int64_t gs_stride, int64_t n_pairs, float* rows_ws,
                           float* drows, float* dw1, float* dv,
                           rs_stream_t stream);

/* One launch per pipelined step (sharded.py pipe_step), run after the
 * step's all-to-all: the owner part of batch t on recv's row-id words
 * (partials -> send's partial words), batch t+1's field route (ids_next ->
 * send's row-id words; ids_next NULL = none) and batch t-1's combine
 * (recv's partial words + dense_prev -> logit_prev; logit_prev NULL = none).
 * recv and send hold world*batch fused records of slot_stride + P words
 * ([row ids | partial]).  The three parts are independent, so one pipelined
 * step is exactly one kernel and one all-to-all.                           */
int rs_shard_fm_pipe(const int32_t* recv, int field_lo, int n_owned,
                     const float* shard, int64_t shard_rows,
                     const float* dense_prev, int64_t dense_stride,
                     float* logit_prev, const void* ids_next, int id_kind,
                     int64_t id_stride, const int64_t* field_offsets,
                     const int64_t* field_vocab, int64_t rows_per_rank,
                     const int32_t* owner_fields, int slot_stride,
                     int32_t* send, int world, int64_t batch, int nd,
                     int n_fields, int k, const float* prepared,
                     const float* w0, int kfm, int* err_flag,
                     rs_stream_t stream);

/* The TWO-DEEP pipelined step with the peer-mapped exchange inside the
 * launch (sharded.py pipe2_step; replaces, for the step, the all-to-all
 * torch.distributed would run before rs_shard_fm_pipe — the lookup sharded is
 * EmbedLayer.call, layer/core.py:273-280).  Launch t = exchange of batch t+1
 * (if `exchange`: this rank's send slot `xsend` = [world][batch] records of
 * [row ids of t+1 | partials of t-1] copied into slot `xslot` of every
 * peer's two-slot mailbox, rs_peer_a2a's ready / full protocol, one step of
 * `peer_state`) | combine of batch t-2 (logit_prev) | owner partials of batch
 * t | field route of batch t+2 (ids_next), the three pipe parts reading
 * `recv` (= this rank's mailbox slot t % 2) and writing `send` (= send slot
 * t % 2).  mailboxes: device array [world] of two-slot mailboxes
 * (rs_peer_mailbox_bytes(world, 2 * batch * R * 4), R = slot_stride +
 * rs_fm_partial_width(kfm)); the launch ends when every peer's block of this
 * step is in this rank's mailbox.  A bounded wait that gives up sets
 * RS_FLAG_TIMEOUT in xerr.  kfm <= 15, <= 32 owned fields, batch * R * 4 a
 * multiple of 16 (else RS_ERR_UNSUPPORTED / RS_ERR_ARG).                    */
int rs_shard_fm_pipe_peer(const int32_t* recv, int32_t* send,
                          const int32_t* xsend, int xslot, int exchange,
                          int field_lo, int n_owned, const float* shard,
                          int64_t shard_rows, const float* dense_prev,
                          int64_t dense_stride, float* logit_prev,
                          const void* ids_next, int id_kind, int64_t id_stride,
                          const int64_t* field_offsets,
                          const int64_t* field_vocab, int64_t rows_per_rank,
                          const int32_t* owner_fields, int slot_stride,
                          int world, int64_t batch, int nd, int n_fields,
                          int k, const float* prepared, const float* w0,
                          int kfm, int* err_flag, void* const* mailboxes,
                          int rank, void* peer_state, int chunks,
                          int64_t spin_limit, int* xerr, rs_stream_t stream);

/* S consecutive batch requests in ONE launch (the headline hot path served
 * back to back: EmbedLayer + concat + FMLayer, layer/core.py:273-280,
 * layer/interaction.py:106-114, per batch as rs_embed_fm_fwd_hm computes it):
 * batch s (s < n_batches) has `batch` samples (the last one last_batch), its
 * ids at ids + s * ids_batch_stride elements (rows id_stride apart), dense at
 * dense + s * dense_batch_stride floats, logits written at logit + s *
 * logit_batch_stride.  Every batch's logits are bit-identical to
 * rs_embed_fm_fwd_hm on that batch alone (same kernel body and tiles).
 * Shapes of the kernarg-metadata kernel only: k in {4, 8, 16}, kfm <= 15,
 * 1..32 fields (host metadata), nd <= 64, int32 / int64 ids, batch <= 8192;
 * min_blocks = 1 or 2 resident workgroups per CU (RS_ERR_ARG otherwise).    */
int rs_embed_fm_fwd_hm_stream(const void* ids, int id_kind, int64_t id_stride,
                              int64_t ids_batch_stride, const float* dense,
                              int64_t dense_stride, int64_t dense_batch_stride,
                              int nd, const float* table,
                              const int64_t* field_offsets_host,
                              const int64_t* field_vocab_host, int n_fields,
                              int k, const float* prepared, const float* w0,
                              int kfm, float* logit,
                              int64_t logit_batch_stride, int64_t batch,
                              int n_batches, int64_t last_batch,
                              int min_blocks, int* err_flag,
                              rs_stream_t stream);

/* FM over pre-gathered rows (sharded path): emb is [B, F*k] in x order.     */
int rs_rows_fm_fwd(const float* emb, const float* dense, int64_t dense_stride,
                   int nd, int n_fields, int k, const float* prepared,
                   const float* w0, int kfm, float* logit, int64_t batch,
                   rs_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RS_CAPI_H */
