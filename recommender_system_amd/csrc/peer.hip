// peer.hip — peer-mapped all-to-all for the row-sharded lookup (sharded.py
// PeerExchange): a rank writes its send blocks straight into its peers'
// receive mailboxes (hipIpc-mapped device memory: loads/stores over xGMI on
// an 8-GPU node), instead of an RCCL all-to-all.  Reference: the lookup being
// sharded is EmbedLayer.call, algorithm/deep_learning/layer/core.py:273-280
// (the reference has no distributed code).
//
// Mailbox of a rank (one uncached device allocation, IPC-exported):
//   data  [world][block_bytes]   block r = what rank r sent me this step
//   ready [world] x 128 B        ready[r] = the last step for which rank r's
//                                mailbox is free (written by rank r at every peer)
//   full  [world] x 128 B        full[r]  = the last step whose block from rank r
//                                is in my data (written by rank r; full-fence mode)
//   chunk [world][chunks] x 8 B  lean mode: [r][c] = the last step whose chunk c
//                                from rank r is in my data (written by that
//                                workgroup of rank r)
// Per-rank local state (ordinary device memory): seq (steps done), a
// per-destination chunk counter, and a completed-workgroup counter.
//
// One launch per exchange, graph-capturable (the step number lives on the
// device: seq = state.seq + 1, advanced by the kernel itself):
//   1. workgroup 0 tells every peer that my mailbox is free for step seq
//      (ready[me] = seq at each peer): the kernels that read the previous
//      step's data ran before this one on my stream;
//   2. workgroup (c, p) requests its first words of chunk c of my block for
//      p (local sources), waits until peer p's mailbox is free for seq (p's
//      ready word in MY mailbox: a local poll), stores the chunk into p's
//      data[me] (16-B stores) and drains them; then
//      - lean mode: sets its own chunk flag [me][c] = seq at p and its done
//        word in my state (plain write-through stores, no shared counter);
//      - full-fence mode: releases at system scope and counts itself on p's
//        chunk counter; the last chunk writer of destination p sets
//        full[me] = seq at p (release store, system scope);
//   3. workgroup 0 waits for every chunk of step seq to be in my mailbox
//      (lean: all [r][c] chunk flags; full-fence: full[r] from every rank r,
//      acquire) and for every workgroup of this launch to be done, then
//      advances state.seq — so the launch completes only when my mailbox
//      holds the whole step, and the next kernel on the stream reads it.
// Every spin is bounded: a wait that gives up sets RS_FLAG_TIMEOUT in the
// error flag and the launch still drains (the host raises RSError).  The
// mailbox is uncached device memory, so no stale L2 line of a previous step
// can be read after a peer's writes.
#include <string.h>

#include "peer.hpp"

namespace rs {

template <bool GATHER>
__global__ __launch_bounds__(256) void peer_a2a_kernel(PeerArgs a) {
  peer_a2a_part<GATHER>(a, blockIdx.x, blockIdx.y);
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_peer_state_bytes(void) { return (int64_t)sizeof(PeerState); }

extern "C" int64_t rs_peer_mailbox_bytes(int world, int64_t block_bytes) {
  if (world < 1 || world > PEER_MAXW || block_bytes < 0 || block_bytes % 16) return -1;
  const int64_t data = ((int64_t)world * block_bytes + 255) / 256 * 256;
  return data + 2 * (int64_t)world * PEER_FLAG_STRIDE + PEER_MAXBLK * 8;
}

extern "C" int rs_peer_alloc(int64_t bytes, void** ptr) {
  RS_REQUIRE(bytes > 0 && ptr, "rs_peer_alloc: bad arguments");
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) {
    set_error("rs_peer_alloc: hipExtMallocWithFlags(uncached) failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  e = hipMemset(p, 0, (size_t)bytes);
  if (e != hipSuccess) {
    (void)hipFree(p);
    set_error("rs_peer_alloc: hipMemset failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  *ptr = p;
  return RS_OK;
}

extern "C" int rs_peer_free(void* ptr) {
  if (!ptr) return RS_OK;
  const hipError_t e = hipFree(ptr);
  if (e != hipSuccess) {
    set_error("rs_peer_free: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  return RS_OK;
}

extern "C" int rs_peer_ipc_handle(void* ptr, void* handle64) {
  RS_REQUIRE(ptr && handle64, "rs_peer_ipc_handle: null pointer");
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e != hipSuccess) {
    set_error("rs_peer_ipc_handle: hipIpcGetMemHandle failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  memcpy(handle64, &h, sizeof(h));
  return RS_OK;
}

extern "C" int rs_peer_ipc_open(const void* handle64, void** ptr) {
  RS_REQUIRE(handle64 && ptr, "rs_peer_ipc_open: null pointer");
  hipIpcMemHandle_t h;
  memcpy(&h, handle64, sizeof(h));
  void* p = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    set_error("rs_peer_ipc_open: hipIpcOpenMemHandle failed: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  *ptr = p;
  return RS_OK;
}

extern "C" int rs_peer_ipc_close(void* ptr) {
  if (!ptr) return RS_OK;
  const hipError_t e = hipIpcCloseMemHandle(ptr);
  if (e != hipSuccess) {
    set_error("rs_peer_ipc_close: %s", hipGetErrorString(e));
    return RS_ERR_HIP;
  }
  return RS_OK;
}

extern "C" int rs_peer_a2a(const void* send, int64_t block_bytes, void* const* mailboxes, int rank, int world,
                           void* state, int chunks, int64_t spin_limit, int* err_flag, rs_stream_t stream) {
  RS_REQUIRE(world >= 1 && world <= PEER_MAXW && rank >= 0 && rank < world, "rs_peer_a2a: bad rank / world");
  RS_REQUIRE(block_bytes >= 0 && block_bytes % 16 == 0, "rs_peer_a2a: block_bytes must be a multiple of 16");
  RS_REQUIRE(mailboxes && state && (block_bytes == 0 || send), "rs_peer_a2a: null pointer");
  RS_REQUIRE(chunks >= 1 && (int64_t)chunks * world <= 1024 && spin_limit >= 1, "rs_peer_a2a: bad chunks / limit");
  PeerArgs a{static_cast<const char*>(send), block_bytes, reinterpret_cast<char* const*>(mailboxes),
             ((int64_t)world * block_bytes + 255) / 256 * 256, static_cast<PeerState*>(state), rank, world, chunks,
             spin_limit, err_flag, nullptr, 0, nullptr, 0, 0, opt(RS_OPT_PEER_FENCES) == 0};
  peer_a2a_kernel<false><<<dim3(chunks, world), 256, 0, as_stream(stream)>>>(a);
  return launch_status("rs_peer_a2a");
}

extern "C" int rs_peer_gather_a2a(const int32_t* ids, int64_t nw, const float* table, int64_t n_rows, int k,
                                  void* const* mailboxes, int rank, int world, void* state, int chunks,
                                  int64_t spin_limit, int* err_flag, rs_stream_t stream) {
  RS_REQUIRE(world >= 1 && world <= PEER_MAXW && rank >= 0 && rank < world, "rs_peer_gather_a2a: bad rank / world");
  RS_REQUIRE(k == 16, "rs_peer_gather_a2a: k must be 16");
  RS_REQUIRE(nw >= 0 && n_rows >= 0 && (uintptr_t)table % 16 == 0, "rs_peer_gather_a2a: bad shape / alignment");
  RS_REQUIRE(mailboxes && state && (nw == 0 || ids) && (n_rows == 0 || table), "rs_peer_gather_a2a: null pointer");
  RS_REQUIRE(chunks >= 1 && (int64_t)chunks * world <= 1024 && spin_limit >= 1,
             "rs_peer_gather_a2a: bad chunks / limit");
  const int64_t block_bytes = nw * 64;
  PeerArgs a{nullptr, block_bytes, reinterpret_cast<char* const*>(mailboxes),
             ((int64_t)world * block_bytes + 255) / 256 * 256, static_cast<PeerState*>(state), rank, world, chunks,
             spin_limit, err_flag, ids, nw, table, n_rows, 0, opt(RS_OPT_PEER_FENCES) == 0};
  peer_a2a_kernel<true><<<dim3(chunks, world), 256, 0, as_stream(stream)>>>(a);
  return launch_status("rs_peer_gather_a2a");
}
