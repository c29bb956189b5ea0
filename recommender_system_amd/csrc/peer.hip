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
//                                is in my data (written by rank r)
// Per-rank local state (ordinary device memory): seq (steps done), a
// per-destination chunk counter, and a completed-workgroup counter.
//
// One launch per exchange, graph-capturable (the step number lives on the
// device: seq = state.seq + 1, advanced by the kernel itself):
//   1. workgroup 0 tells every peer that my mailbox is free for step seq
//      (ready[me] = seq at each peer): the kernels that read the previous
//      step's data ran before this one on my stream;
//   2. workgroup (c, p) waits until peer p's mailbox is free for seq (p's
//      ready word in MY mailbox: a local poll), copies
//      chunk c of my block for p into p's data[me] (16-B stores), drains its
//      stores, releases at system scope and counts itself on p's chunk
//      counter; the last chunk writer of destination p sets full[me] = seq
//      at p (release store, system scope);
//   3. workgroup 0 waits for full[r] == seq from every rank r (acquire) and
//      for every workgroup of this launch to have counted itself, then
//      advances state.seq — so the launch completes only when my mailbox
//      holds the whole step, and the next kernel on the stream reads it.
// Every spin is bounded: a wait that gives up sets RS_FLAG_TIMEOUT in the
// error flag and the launch still drains (the host raises RSError).  The
// mailbox is uncached device memory, so no stale L2 line of a previous step
// can be read after a peer's writes.
#include <string.h>

#include "rs_common.hpp"

namespace rs {

struct PeerState {  // per-rank local state, rs_peer_state_bytes() bytes, zeroed by the caller once
  unsigned long long seq;
  unsigned int total;
  unsigned int pad[29];
  unsigned int cnt[64];  // per destination: chunks written this step
};
constexpr int PEER_MAXW = 64;
constexpr int PEER_FLAG_STRIDE = 128;  // bytes: each flag on its own line

struct PeerArgs {
  const char* send;      // [world][block_bytes], local (GATHER: unused)
  int64_t block_bytes;   // multiple of 16
  char* const* mbox;     // device array [world]: every rank's mailbox base (mine at [rank])
  int64_t data_bytes;    // world * block_bytes, rounded up to 256 (offset of the flags)
  PeerState* st;
  int rank, world, chunks;  // chunks per destination (grid = chunks x world)
  int64_t spin_limit;
  int* err;
  // GATHER (rs_peer_gather_a2a): block p is gathered on the fly — row ids[p][i]
  // of the local table shard (k = 16 floats, -1 = a zero row) for every word i
  const int32_t* ids;  // [world][nw] local row ids (the requests each peer sent me)
  int64_t nw;
  const float* table;
  int64_t n_rows;
};

__device__ __forceinline__ unsigned long long* peer_flag(char* mbox, int64_t data_bytes, int which, int world,
                                                         int r) {
  return reinterpret_cast<unsigned long long*>(mbox + data_bytes +
                                               ((int64_t)which * world + r) * PEER_FLAG_STRIDE);
}

// bounded wait until *f >= v (one lane); false on timeout
__device__ __forceinline__ bool peer_wait_ge(unsigned long long* f, unsigned long long v, int64_t limit) {
  for (int64_t i = 0; i < limit; ++i) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= v) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= v;
}

template <bool GATHER>
__global__ __launch_bounds__(256) void peer_a2a_kernel(PeerArgs a) {
  const int c = blockIdx.x, p = blockIdx.y;
  const unsigned long long seq = a.st->seq + 1;
  __shared__ int ok_s;
  bool ok = true;
  // 1. my mailbox is free for this step: tell every peer
  if (c == 0 && p == 0 && threadIdx.x < (unsigned)a.world)
    __hip_atomic_store(peer_flag(a.mbox[threadIdx.x], a.data_bytes, 0, a.world, a.rank), seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 2. peer p's mailbox free for this step? (p's step 1 wrote ready[p] in MY mailbox: a local poll)
  if (threadIdx.x == 0) ok_s = peer_wait_ge(peer_flag(a.mbox[a.rank], a.data_bytes, 0, a.world, p), seq, a.spin_limit);
  __syncthreads();
  ok = ok_s != 0;
  if (ok) {
    const int64_t per = (a.block_bytes / 16 + a.chunks - 1) / a.chunks;  // 16-B words per chunk
    const int64_t w0 = (int64_t)c * per, w1 = min<int64_t>(w0 + per, a.block_bytes / 16);
    floatx4* dst = reinterpret_cast<floatx4*>(a.mbox[p] + (int64_t)a.rank * a.block_bytes);
    if constexpr (GATHER) {
      // 4 lanes per 64-B row: row ids[p][i >> 2], quarter i & 3 (non-temporal: read once)
      const int32_t* rid = a.ids + (int64_t)p * a.nw;
      bool bad = false;
      for (int64_t i = w0 + threadIdx.x; i < w1; i += blockDim.x) {
        const int64_t r = rid[i >> 2];
        floatx4 x = {0.f, 0.f, 0.f, 0.f};
        if (r >= 0 && r < a.n_rows) x = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.table + r * 16) + (i & 3));
        else bad |= r != -1;
        dst[i] = x;
      }
      if (__any(bad) && (threadIdx.x & 63) == 0) flag_error(a.err);
    } else {
      const floatx4* src = reinterpret_cast<const floatx4*>(a.send + (int64_t)p * a.block_bytes);
      for (int64_t i = w0 + threadIdx.x; i < w1; i += blockDim.x) dst[i] = src[i];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (!ok) flag_error(a.err, RS_FLAG_TIMEOUT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: my chunk before the count / flag
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(&a.st->cnt[p], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)a.chunks - 1) {
      a.st->cnt[p] = 0;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      __hip_atomic_store(peer_flag(a.mbox[p], a.data_bytes, 1, a.world, a.rank), seq, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_fetch_add(&a.st->total, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  // 3. workgroup 0: the whole step in my mailbox, every workgroup counted
  if (c == 0 && p == 0) {
    bool done = true;
    if (threadIdx.x < (unsigned)a.world)
      done = peer_wait_ge(peer_flag(a.mbox[a.rank], a.data_bytes, 1, a.world, threadIdx.x), seq, a.spin_limit);
    if (threadIdx.x == 0) {
      const unsigned nblk = (unsigned)a.chunks * (unsigned)a.world;
      int64_t i = 0;
      for (; i < a.spin_limit && __hip_atomic_load(&a.st->total, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < nblk;
           ++i)
        __builtin_amdgcn_s_sleep(2);
      done = done && i < a.spin_limit;
    }
    if (!done) flag_error(a.err, RS_FLAG_TIMEOUT);
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      a.st->total = 0;
      a.st->seq = seq;
    }
  }
}

}  // namespace rs

using namespace rs;

extern "C" int64_t rs_peer_state_bytes(void) { return (int64_t)sizeof(PeerState); }

extern "C" int64_t rs_peer_mailbox_bytes(int world, int64_t block_bytes) {
  if (world < 1 || world > PEER_MAXW || block_bytes < 0 || block_bytes % 16) return -1;
  const int64_t data = ((int64_t)world * block_bytes + 255) / 256 * 256;
  return data + 2 * (int64_t)world * PEER_FLAG_STRIDE;
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
             spin_limit, err_flag, nullptr, 0, nullptr, 0};
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
             spin_limit, err_flag, ids, nw, table, n_rows};
  peer_a2a_kernel<true><<<dim3(chunks, world), 256, 0, as_stream(stream)>>>(a);
  return launch_status("rs_peer_gather_a2a");
}
