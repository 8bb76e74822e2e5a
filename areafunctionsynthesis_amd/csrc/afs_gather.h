// afs_gather.h -- utterance shards and the audio gather to rank 0, independent of the
// transport (host-only code: libafs.so drives it over RCCL, tests/cpp/gather_main.cpp over an
// in-process loopback).
//
// The batch is the only axis that splits: rank r owns a contiguous block of
// utterances and there is no exchange while they synthesize.  The one collective is the
// gather of the finished audio to rank 0, in the reference's output format (int16 Signal16,
// Synthesizer.cpp:955-973): rank 0 receives every block at its utterance offset, so the
// gathered buffer is exactly the [B][T] array one device would have produced.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace afs {

// Contiguous block of `rank` when `total` items are split over `world` ranks: the first
// total % world ranks take one more item.
inline void shard_range(int64_t total, int32_t world, int32_t rank, int64_t *first, int64_t *count) {
  const int64_t q = total / world, r = total % world;
  *count = q + (rank < r ? 1 : 0);
  *first = (int64_t)rank * q + (rank < r ? rank : r);
}

// Gather `bytes` from every rank into root_out (rank 0 only) at the byte offsets
// prefix(root_bytes).  T provides rank(), world(), group_start(), group_end(),
// send(const void*, size_t, int peer), recv(void*, size_t, int peer),
// copy_local(void *dst, const void *src, size_t) and returns 0 / an error code from each.
// root_bytes: rank 0's view of every rank's byte count (null: all equal to `bytes`).
template <class T>
int gather_to_root(T &t, const void *local, size_t bytes, void *root_out, const size_t *root_bytes) {
  const int world = t.world(), rank = t.rank();
  if (world == 1) return bytes ? t.copy_local(root_out, local, bytes) : 0;
  int e = t.group_start();
  if (e) return e;
  if (rank == 0) {
    size_t off = 0;
    for (int p = 0; p < world && !e; ++p) {
      const size_t n = root_bytes ? root_bytes[p] : bytes;
      char *dst = static_cast<char *>(root_out) + off;
      if (n) e = p == 0 ? t.copy_local(dst, local, n) : t.recv(dst, n, p);
      off += n;
    }
  } else if (bytes) {
    e = t.send(local, bytes, 0);
  }
  const int e2 = t.group_end();
  return e ? e : e2;
}

// rank 0's byte counts of a gather of `per_item` bytes per utterance when `total` utterances
// are sharded with shard_range over `world` ranks
inline std::vector<size_t> shard_bytes(int64_t total, int32_t world, size_t per_item) {
  std::vector<size_t> v((size_t)world);
  for (int r = 0; r < world; ++r) {
    int64_t first, count;
    shard_range(total, world, r, &first, &count);
    v[(size_t)r] = (size_t)count * per_item;
  }
  return v;
}

}  // namespace afs
