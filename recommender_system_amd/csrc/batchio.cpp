// batchio.cpp — the input producer's on-disk format.
//
// The reference hands the model X[N, 13+26] float64 with the label-encoded
// sparse ids packed as floats (utils/dataset.py:36-65: fillna -> MinMaxScaler
// -> LabelEncoder -> .values), which Keras casts to float32 (ids exact only
// below 2^24) and back to int32 inside Embedding.  RSCB keeps the same
// information in the GPU path's own layout, so a batch is three contiguous
// slabs that go to HBM with three DMA copies and straight into the kernels:
//
//   header (4 KiB): magic "RSCB0001", version, n_rows, n_dense, n_sparse,
//                   id_bytes (4 | 8), section offsets, then n_sparse field
//                   vocab sizes (features_dict's nunique()+1) and one-hot
//                   field offsets (sum of the preceding vocab sizes)
//   dense  [n_rows, n_dense]  float32 (MinMax-scaled)        4 KiB aligned
//   ids    [n_rows, n_sparse] int32 | int64 label codes      4 KiB aligned
//   labels [n_rows]           float32                        4 KiB aligned
//
// Host-only code (no device calls): the writer validates every id against
// its field's vocab (the reference would raise at lookup time); the reader
// mmaps the file and copies row ranges into caller buffers (pinned host
// memory for the H2D stage), splitting large copies over threads.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "rs_batchio.h"
#include "rs_common.hpp"

namespace {

constexpr char kMagic[8] = {'R', 'S', 'C', 'B', '0', '0', '0', '1'};
constexpr int64_t kHeader = 4096;
constexpr int kMaxSparse = (kHeader - 128) / 16;

struct Header {
  char magic[8];
  uint32_t version;
  uint32_t n_dense;
  uint32_t n_sparse;
  uint32_t id_bytes;
  uint64_t n_rows;
  uint64_t off_dense, off_ids, off_labels, file_size;
};
static_assert(sizeof(Header) <= 128, "RSCB header");

int64_t align4k(int64_t x) { return (x + 4095) / 4096 * 4096; }

struct File {
  int fd = -1;
  uint8_t* base = nullptr;
  size_t size = 0;
  Header h{};
  std::vector<int64_t> vocab, offs;
};

bool write_all(int fd, const void* p, size_t n, int64_t off) {
  const uint8_t* c = static_cast<const uint8_t*>(p);
  while (n) {
    const ssize_t w = pwrite(fd, c, n, off);
    if (w <= 0) return false;
    c += w;
    off += w;
    n -= (size_t)w;
  }
  return true;
}

// memcpy split over up to 8 threads (>= 1 MiB each) for large slabs
// (page cache -> pinned host memory)
void par_copy(void* dst, const void* src, size_t n) {
  const size_t chunk = 1u << 20;
  const int nt = (int)std::min<size_t>(8, (n + chunk - 1) / chunk);
  if (nt <= 1) {
    memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> ts;
  const size_t per = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    const size_t o = (size_t)t * per;
    if (o >= n) break;
    ts.emplace_back([=] { memcpy(static_cast<uint8_t*>(dst) + o, static_cast<const uint8_t*>(src) + o,
                                 std::min(per, n - o)); });
  }
  for (auto& t : ts) t.join();
}

}  // namespace

extern "C" int rs_cb_write(const char* path, int64_t n_rows, int n_dense, int n_sparse, int id_bytes,
                           const float* dense, const void* ids, const float* labels, const int64_t* field_vocab,
                           const int64_t* field_offsets) {
  RS_REQUIRE(path && n_rows >= 0 && n_dense >= 0 && n_sparse >= 0 && n_sparse <= kMaxSparse &&
                 (id_bytes == 4 || id_bytes == 8),
             "rs_cb_write: bad shape (n_sparse <= %d, id_bytes 4 or 8)", kMaxSparse);
  RS_REQUIRE((n_dense == 0 || dense || n_rows == 0) && (n_sparse == 0 || (ids && field_vocab) || n_rows == 0),
             "rs_cb_write: null pointer");
  for (int c = 0; c < n_sparse; ++c) RS_REQUIRE(field_vocab[c] >= 1, "rs_cb_write: field %d has vocab < 1", c);
  if (id_bytes == 4)
    for (int c = 0; c < n_sparse; ++c)
      RS_REQUIRE(field_vocab[c] <= INT32_MAX, "rs_cb_write: field %d vocab needs 64-bit ids", c);
  for (int64_t r = 0; r < n_rows; ++r)
    for (int c = 0; c < n_sparse; ++c) {
      const int64_t id = id_bytes == 4 ? static_cast<const int32_t*>(ids)[r * n_sparse + c]
                                       : static_cast<const int64_t*>(ids)[r * n_sparse + c];
      RS_REQUIRE(id >= 0 && id < field_vocab[c], "rs_cb_write: row %lld field %d id %lld outside [0, %lld)",
                 (long long)r, c, (long long)id, (long long)field_vocab[c]);
    }
  Header h{};
  memcpy(h.magic, kMagic, 8);
  h.version = 1;
  h.n_dense = (uint32_t)n_dense;
  h.n_sparse = (uint32_t)n_sparse;
  h.id_bytes = (uint32_t)id_bytes;
  h.n_rows = (uint64_t)n_rows;
  h.off_dense = kHeader;
  h.off_ids = align4k(h.off_dense + n_rows * n_dense * 4);
  h.off_labels = align4k(h.off_ids + n_rows * n_sparse * id_bytes);
  h.file_size = align4k(h.off_labels + n_rows * 4);
  std::vector<uint8_t> head(kHeader, 0);
  memcpy(head.data(), &h, sizeof(h));
  std::vector<int64_t> offs(n_sparse);
  for (int c = 0; c < n_sparse; ++c)
    offs[c] = field_offsets ? field_offsets[c] : (c ? offs[c - 1] + field_vocab[c - 1] : 0);
  memcpy(head.data() + 128, field_vocab, n_sparse * 8);
  memcpy(head.data() + 128 + n_sparse * 8, offs.data(), n_sparse * 8);
  const int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
  RS_REQUIRE(fd >= 0, "rs_cb_write: cannot create %s: %s", path, strerror(errno));
  bool ok = ftruncate(fd, (off_t)h.file_size) == 0 && write_all(fd, head.data(), kHeader, 0) &&
            write_all(fd, dense, n_rows * n_dense * 4, h.off_dense) &&
            write_all(fd, ids, n_rows * n_sparse * id_bytes, h.off_ids) &&
            (!labels || write_all(fd, labels, n_rows * 4, h.off_labels));
  ok = (close(fd) == 0) && ok;
  RS_REQUIRE(ok, "rs_cb_write: write to %s failed", path);
  return RS_OK;
}

extern "C" void* rs_cb_open(const char* path) {
  if (!path) {
    rs::set_error("rs_cb_open: null path");
    return nullptr;
  }
  const int fd = open(path, O_RDONLY);
  if (fd < 0) {
    rs::set_error("rs_cb_open: cannot open %s: %s", path, strerror(errno));
    return nullptr;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < kHeader) {
    close(fd);
    rs::set_error("rs_cb_open: %s is not an RSCB file (too short)", path);
    return nullptr;
  }
  void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    close(fd);
    rs::set_error("rs_cb_open: mmap %s failed: %s", path, strerror(errno));
    return nullptr;
  }
  auto* f = new File;
  f->fd = fd;
  f->base = static_cast<uint8_t*>(m);
  f->size = (size_t)st.st_size;
  memcpy(&f->h, f->base, sizeof(Header));
  const Header& h = f->h;
  // section extents in checked arithmetic: a crafted header must not wrap a
  // product past the bounds checks (rs_cb_read copies straight from the map)
  auto sect_end = [](uint64_t off, uint64_t rows, uint64_t cols, uint64_t width, uint64_t* end) {
    uint64_t n = 0;
    return !__builtin_mul_overflow(rows, cols, &n) && !__builtin_mul_overflow(n, width, &n) &&
           !__builtin_add_overflow(off, n, end);
  };
  uint64_t end_dense = 0, end_ids = 0, end_labels = 0;
  const bool aligned = h.off_dense % kHeader == 0 && h.off_ids % kHeader == 0 && h.off_labels % kHeader == 0;
  const bool ok = memcmp(h.magic, kMagic, 8) == 0 && h.version == 1 && (h.id_bytes == 4 || h.id_bytes == 8) &&
                  h.n_sparse <= (uint32_t)kMaxSparse && h.file_size <= f->size && aligned &&
                  h.off_dense >= (uint64_t)kHeader &&
                  sect_end(h.off_dense, h.n_rows, h.n_dense, 4, &end_dense) && end_dense <= h.off_ids &&
                  sect_end(h.off_ids, h.n_rows, h.n_sparse, h.id_bytes, &end_ids) && end_ids <= h.off_labels &&
                  sect_end(h.off_labels, h.n_rows, 1, 4, &end_labels) && end_labels <= h.file_size;
  if (!ok) {
    rs_cb_close(f);
    rs::set_error("rs_cb_open: %s: bad RSCB header", path);
    return nullptr;
  }
  f->vocab.resize(h.n_sparse);
  f->offs.resize(h.n_sparse);
  memcpy(f->vocab.data(), f->base + 128, h.n_sparse * 8);
  memcpy(f->offs.data(), f->base + 128 + h.n_sparse * 8, h.n_sparse * 8);
  madvise(f->base, f->size, MADV_SEQUENTIAL);
  return f;
}

extern "C" int rs_cb_info(void* handle, int64_t* n_rows, int* n_dense, int* n_sparse, int* id_bytes,
                          int64_t* field_vocab, int64_t* field_offsets) {
  RS_REQUIRE(handle, "rs_cb_info: null handle");
  const File* f = static_cast<const File*>(handle);
  if (n_rows) *n_rows = (int64_t)f->h.n_rows;
  if (n_dense) *n_dense = (int)f->h.n_dense;
  if (n_sparse) *n_sparse = (int)f->h.n_sparse;
  if (id_bytes) *id_bytes = (int)f->h.id_bytes;
  if (field_vocab) memcpy(field_vocab, f->vocab.data(), f->vocab.size() * 8);
  if (field_offsets) memcpy(field_offsets, f->offs.data(), f->offs.size() * 8);
  return RS_OK;
}

extern "C" int rs_cb_read(void* handle, int64_t row0, int64_t count, float* dense, void* ids, float* labels) {
  RS_REQUIRE(handle, "rs_cb_read: null handle");
  const File* f = static_cast<const File*>(handle);
  const Header& h = f->h;
  RS_REQUIRE(row0 >= 0 && count >= 0 && (uint64_t)(row0 + count) <= h.n_rows,
             "rs_cb_read: rows [%lld, %lld) outside [0, %llu)", (long long)row0, (long long)(row0 + count),
             (unsigned long long)h.n_rows);
  if (dense) par_copy(dense, f->base + h.off_dense + row0 * h.n_dense * 4, count * h.n_dense * 4);
  if (ids) par_copy(ids, f->base + h.off_ids + row0 * h.n_sparse * h.id_bytes, count * h.n_sparse * h.id_bytes);
  if (labels) par_copy(labels, f->base + h.off_labels + row0 * 4, count * 4);
  return RS_OK;
}

extern "C" void rs_cb_close(void* handle) {
  File* f = static_cast<File*>(handle);
  if (!f) return;
  if (f->base) munmap(f->base, f->size);
  if (f->fd >= 0) close(f->fd);
  delete f;
}
