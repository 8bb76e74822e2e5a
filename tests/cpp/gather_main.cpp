// The shard / gather logic of afs_gather.h (what libafs.so runs over RCCL) over an in-process
// loopback transport: one thread per rank, sends land in mailboxes that rank 0 drains.
// Prints "gather-ok" when every configuration reassembles the batch exactly.
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "afs_gather.h"

struct Mailboxes {
  std::mutex m;
  std::condition_variable cv;
  std::map<std::pair<int, int>, std::vector<char>> box;  // (from, to) -> bytes
};

struct Loopback {
  Mailboxes *mb;
  int r, w;
  int groups = 0;
  int rank() const { return r; }
  int world() const { return w; }
  int group_start() { ++groups; return 0; }
  int group_end() { return groups-- > 0 ? 0 : 1; }
  int send(const void *p, size_t n, int peer) {
    std::lock_guard<std::mutex> g(mb->m);
    auto &b = mb->box[{r, peer}];
    if (!b.empty()) return 2;  // one message per pair and gather
    b.assign((const char *)p, (const char *)p + n);
    mb->cv.notify_all();
    return 0;
  }
  int recv(void *p, size_t n, int peer) {
    std::unique_lock<std::mutex> g(mb->m);
    mb->cv.wait(g, [&] { return !mb->box[{peer, r}].empty(); });
    auto &b = mb->box[{peer, r}];
    if (b.size() != n) return 3;
    std::memcpy(p, b.data(), n);
    b.clear();
    return 0;
  }
  int copy_local(void *d, const void *s, size_t n) { std::memcpy(d, s, n); return 0; }
};

// B utterances of T int16 samples, value = f(u, t); every rank synthesizes its shard
static int16_t sample(int64_t u, int64_t t) { return (int16_t)((u * 7919 + t * 31) % 65521 - 32760); }

static bool run(int world, int64_t B, int64_t T) {
  // shards cover [0, B) exactly once, in order
  int64_t next = 0;
  for (int r = 0; r < world; ++r) {
    int64_t f, n;
    afs::shard_range(B, world, r, &f, &n);
    if (f != next || n < 0) return false;
    next = f + n;
  }
  if (next != B) return false;
  Mailboxes mb;
  std::vector<int16_t> root((size_t)(B * T), 0);
  const std::vector<size_t> rb = afs::shard_bytes(B, world, (size_t)T * sizeof(int16_t));
  std::vector<int> err((size_t)world, 0);
  std::vector<std::thread> th;
  for (int r = 0; r < world; ++r)
    th.emplace_back([&, r] {
      int64_t f, n;
      afs::shard_range(B, world, r, &f, &n);
      std::vector<int16_t> local((size_t)(n * T));
      for (int64_t u = 0; u < n; ++u)
        for (int64_t t = 0; t < T; ++t) local[(size_t)(u * T + t)] = sample(f + u, t);
      Loopback lb{&mb, r, world};
      err[(size_t)r] = afs::gather_to_root(lb, local.data(), local.size() * sizeof(int16_t),
                                           r == 0 ? root.data() : nullptr, r == 0 ? rb.data() : nullptr);
    });
  for (auto &t : th) t.join();
  for (int e : err)
    if (e) return false;
  for (int64_t u = 0; u < B; ++u)
    for (int64_t t = 0; t < T; ++t)
      if (root[(size_t)(u * T + t)] != sample(u, t)) return false;
  return true;
}

int main() {
  const int cfg[][3] = {{1, 5, 7}, {2, 6, 11}, {2, 7, 3}, {3, 10, 5}, {4, 3, 9}, {8, 65, 4}, {8, 8, 1}};
  for (const auto &c : cfg)
    if (!run(c[0], c[1], c[2])) {
      std::printf("gather-fail world=%d B=%d T=%d\n", c[0], c[1], c[2]);
      return 1;
    }
  std::printf("gather-ok\n");
  return 0;
}
