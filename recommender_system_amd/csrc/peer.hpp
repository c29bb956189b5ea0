// peer.hpp — the peer-mapped exchange's device part, shared by the standalone
// exchange (peer.hip: rs_peer_a2a / rs_peer_gather_a2a) and the two-deep
// pipelined sharded FM step that runs the exchange of batch t+1 inside batch
// t's pipe launch (embed_fm.hip: rs_shard_fm_pipe_peer).  The protocol and
// the mailbox layout are described at the top of peer.hip.
#pragma once
#include "rs_common.hpp"

namespace rs {

struct PeerState {  // per-rank local state, rs_peer_state_bytes() bytes, zeroed by the caller once
  unsigned long long seq;
  unsigned int total;
  unsigned int pad[29];
  unsigned int cnt[64];  // per destination: chunks written this step (full-fence mode)
  unsigned long long done[1024];  // lean mode: [p][c] = the last step workgroup (c, p) finished
};
constexpr int PEER_MAXW = 64;
constexpr int PEER_FLAG_STRIDE = 128;  // bytes: each flag on its own line

struct PeerArgs {
  const char* send;      // [world][block_bytes], local (GATHER: unused)
  int64_t block_bytes;   // multiple of 16
  char* const* mbox;     // device array [world]: every rank's mailbox base (mine at [rank])
  int64_t data_bytes;    // offset of the flags in a mailbox (its data region, rounded up to 256)
  PeerState* st;
  int rank, world, chunks;  // chunks per destination (exchange workgroups = chunks x world)
  int64_t spin_limit;
  int* err;
  // GATHER (rs_peer_gather_a2a): block p is gathered on the fly — row ids[p][i]
  // of the local table shard (k = 16 floats, -1 = a zero row) for every word i
  const int32_t* ids;  // [world][nw] local row ids (the requests each peer sent me)
  int64_t nw;
  const float* table;
  int64_t n_rows;
  // offset of this step's [world][block_bytes] region inside every mailbox's
  // data (0 for the one-slot exchange; slot * world * block_bytes for the
  // two-slot mailboxes of the two-deep pipelined step)
  int64_t slot_off;
  // 0: every count and flag behind a system-scope release (buffer_wbl2) and
  // acquire (buffer_inv) — the whole L2 written back / invalidated several
  // times per workgroup; 1 (lean): the data stores themselves write through
  // (sc0 sc1: nothing of the step can sit dirty in any L2), so s_waitcnt
  // vmcnt(0) orders them before relaxed counts and write-through flags, and
  // no cache maintenance runs beside the launch's other work.  At world 1
  // (lean) the mailbox is ordinary device memory (sharded.PeerExchange: no
  // peer, nothing crosses a device) and the data stores are plain: only the
  // next kernels on this stream read them (kernel-boundary coherence); the
  // flags stay write-through
  int lean;
};

__device__ __forceinline__ unsigned long long* peer_flag(char* mbox, int64_t data_bytes, int which, int world,
                                                         int r) {
  return reinterpret_cast<unsigned long long*>(mbox + data_bytes +
                                               ((int64_t)which * world + r) * PEER_FLAG_STRIDE);
}

// lean mode's chunk flags: [r][c] = the last step whose chunk c from rank r is
// in this mailbox (8 B each, after the ready / full flags; at most 1024)
constexpr int PEER_MAXBLK = 1024;
__device__ __forceinline__ unsigned long long* peer_chunk_flag(char* mbox, int64_t data_bytes, int world, int i) {
  return reinterpret_cast<unsigned long long*>(mbox + data_bytes + 2 * (int64_t)world * PEER_FLAG_STRIDE) + i;
}

// bounded wait until *f >= v (one lane); false on timeout
__device__ __forceinline__ bool peer_wait_ge(unsigned long long* f, unsigned long long v, int64_t limit) {
  for (int64_t i = 0; i < limit; ++i) {
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= v) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= v;
}

// One exchange workgroup: chunk c of my block for destination p (workgroup
// (0, 0) also publishes my mailbox's readiness and, last, waits for the whole
// step to have landed in my mailbox and advances the step counter).  Any block
// size that is a multiple of 64 and >= world; every thread of the workgroup
// must call it.
template <bool GATHER>
__device__ __forceinline__ void peer_a2a_part(const PeerArgs& a, int c, int p) {
  const unsigned long long seq = a.st->seq + 1;
  __shared__ int ok_s;
  bool ok = true;
  // 1. my mailbox is free for this step: tell every peer
  // (lean: relaxed — the kernels that read my mailbox ran before this launch)
  if (c == 0 && p == 0 && threadIdx.x < (unsigned)a.world) {
    if (a.lean)
      __hip_atomic_store(peer_flag(a.mbox[threadIdx.x], a.data_bytes, 0, a.world, a.rank), seq, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    else
      __hip_atomic_store(peer_flag(a.mbox[threadIdx.x], a.data_bytes, 0, a.world, a.rank), seq, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // My chunk's first PU words per thread are requested BEFORE the handshake
  // below: the sources (my send block / my table shard and the row ids peers
  // sent me) are local and were written by earlier kernels on this stream, so
  // only the stores into peer p's mailbox wait for its ready flag, and the
  // flag's trip overlaps the loads' (one word per thread per pass left each
  // thread one dependent HBM trip per word).  GATHER: 4 lanes per 64-B row —
  // row ids[p][i >> 2], quarter i & 3, non-temporal (read once).
  constexpr int PU = 8;
  const int64_t per = (a.block_bytes / 16 + a.chunks - 1) / a.chunks;  // 16-B words per chunk
  const int64_t w0 = (int64_t)c * per, w1 = min<int64_t>(w0 + per, a.block_bytes / 16);
  floatx4* dst = reinterpret_cast<floatx4*>(a.mbox[p] + a.slot_off + (int64_t)a.rank * a.block_bytes);
  const int32_t* rid = GATHER ? a.ids + (int64_t)p * a.nw : nullptr;
  const floatx4* src = GATHER ? nullptr : reinterpret_cast<const floatx4*>(a.send + (int64_t)p * a.block_bytes);
  bool bad = false;
  auto fetch = [&](int64_t base, floatx4 (&x)[PU]) {
    if constexpr (GATHER) {
      int64_t r[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int64_t i = base + (int64_t)u * blockDim.x;
        r[u] = i < w1 ? rid[i >> 2] : -1;
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int64_t i = base + (int64_t)u * blockDim.x;
        x[u] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (r[u] >= 0 && r[u] < a.n_rows)
          x[u] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.table + r[u] * 16) + (i & 3));
        else
          bad |= r[u] != -1;
      }
    } else {
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int64_t i = base + (int64_t)u * blockDim.x;
        x[u] = i < w1 ? src[i] : floatx4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto put = [&](int64_t base, const floatx4 (&x)[PU]) {
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i >= w1) break;
      if (a.lean && a.world > 1) {
        // write-through stores (system scope, relaxed: sc0 sc1), 8 B each (see
        // PeerArgs::lean; world 1: ordinary memory, plain stores)
        unsigned long long* d8 = reinterpret_cast<unsigned long long*>(dst + i);
        __hip_atomic_store(d8, __builtin_bit_cast(unsigned long long, floatx2{x[u][0], x[u][1]}), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(d8 + 1, __builtin_bit_cast(unsigned long long, floatx2{x[u][2], x[u][3]}),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        dst[i] = x[u];
      }
    }
  };
  int64_t base = w0 + threadIdx.x;
  floatx4 x[PU];
  fetch(base, x);
  // 2. peer p's mailbox free for this step? (p's step 1 wrote ready[p] in MY mailbox: a local poll)
  if (threadIdx.x == 0) ok_s = peer_wait_ge(peer_flag(a.mbox[a.rank], a.data_bytes, 0, a.world, p), seq, a.spin_limit);
  __syncthreads();
  ok = ok_s != 0;
  if (ok) {
    for (;;) {
      put(base, x);
      base += (int64_t)PU * blockDim.x;
      if (base >= w1) break;
      fetch(base, x);
    }
  }
  if (GATHER && __any(bad) && (threadIdx.x & 63) == 0) flag_error(a.err);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (a.lean) {
    // every store of this workgroup is complete (write-through, waited for):
    // its own done word at p (chunk flag [me][c], write-through) and locally
    // (state.done[p][c]) — plain stores to words nobody else writes: the
    // chunks x world counter atomics this replaces were serialised at one
    // address each (~5 us of a 6.8 MB gather exchange at 256 workgroups)
    if (threadIdx.x == 0) {
      if (!ok) flag_error(a.err, RS_FLAG_TIMEOUT);
      __hip_atomic_store(peer_chunk_flag(a.mbox[p], a.data_bytes, a.world, a.rank * a.chunks + c), seq,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&a.st->done[p * a.chunks + c], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // 3. workgroup 0: every chunk of the step in my mailbox (the [r][c] flags
    // there) and every workgroup of this launch done (so all of them read
    // state.seq before it advances)
    if (c == 0 && p == 0) {
      const int nblk = a.chunks * a.world;
      bool done = true;
      for (int i = threadIdx.x; i < nblk; i += blockDim.x) {
        done = done && peer_wait_ge(peer_chunk_flag(a.mbox[a.rank], a.data_bytes, a.world, i), seq, a.spin_limit);
        int64_t t = 0;
        for (; t < a.spin_limit && __hip_atomic_load(&a.st->done[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < seq;
             ++t)
          __builtin_amdgcn_s_sleep(2);
        done = done && t < a.spin_limit;
      }
      if (!done) flag_error(a.err, RS_FLAG_TIMEOUT);
      __syncthreads();
      if (threadIdx.x == 0) a.st->seq = seq;
    }
    return;
  }
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
      for (; i < a.spin_limit && __hip_atomic_load(&a.st->total, a.lean ? __ATOMIC_RELAXED : __ATOMIC_ACQUIRE,
                                                   __HIP_MEMORY_SCOPE_AGENT) < nblk;
           ++i)
        __builtin_amdgcn_s_sleep(2);
      done = done && i < a.spin_limit;
    }
    if (!done) flag_error(a.err, RS_FLAG_TIMEOUT);
    __syncthreads();
    if (threadIdx.x == 0) {
      // (lean: the mailbox is uncached memory, read by the next kernels on
      // this stream — nothing of it can be stale in this device's L2)
      if (!a.lean) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      a.st->total = 0;
      a.st->seq = seq;
    }
  }
}

}  // namespace rs
