// afs_comm.cpp -- several GPUs: utterance shards and the RCCL gather of the int16 audio
// (include/afs.h, "Several GPUs").  Host orchestration only; the synthesis is afs_synthesize
// on each device and the only collective is the gather (afs_gather.h) of the finished audio.
//
// librccl.so.1 is opened on first use (dlopen, local symbols), so single-GPU callers carry no
// dependency on it and a process that already holds another RCCL copy (PyTorch's) keeps both
// apart.
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "afs_audio.h"
#include "afs_ctx.h"
#include "afs_gather.h"

struct afs_comm {
  afs_ctx *ctx = nullptr;
  ncclComm_t nc = nullptr;
  int rank = 0, world = 1;
  hipStream_t cs = nullptr;  // the gathers' own stream
  hipEvent_t ready = nullptr, done = nullptr;
  bool pending = false;      // a gather was queued since the last fence
  bool aborted = false;      // the communicator was aborted after a failed group (comm_abort)
  // a timing event pair on the comm stream around every gather (afs_comm_gather_times): the
  // pool grows to the gathers in flight between two reads
  std::vector<hipEvent_t> tev;
  size_t tev_used = 0;
  hipEvent_t t_open = nullptr;  // the gather being queued: its start event
  double gather_ms = 0.0;       // summed over the gathers read so far
  int32_t gathers = 0;
};

namespace {

struct Rccl {
  void *h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char *(*GetErrorString)(ncclResult_t) = nullptr;
  bool ok = false;
  std::string why;
};

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.h) break;
    }
    if (!r.h) {
      r.why = std::string("cannot load librccl.so.1: ") + dlerror();
      return;
    }
    auto sym = [&](auto &f, const char *name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(r.h, name));
      if (!f && r.why.empty()) r.why = std::string("librccl lacks ") + name;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommInitAll, "ncclCommInitAll");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.CommAbort, "ncclCommAbort");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    r.ok = r.why.empty();
  });
  return r;
}

// afs_gather.h's transport over one RCCL communicator, on the comm's stream
struct RcclTransport {
  afs_comm *c;
  int rank() const { return c->rank; }
  int world() const { return c->world; }
  int group_start() { return (int)rccl().GroupStart(); }
  int group_end() { return (int)rccl().GroupEnd(); }
  int send(const void *p, size_t n, int peer) { return (int)rccl().Send(p, n, ncclUint8, peer, c->nc, c->cs); }
  int recv(void *p, size_t n, int peer) { return (int)rccl().Recv(p, n, ncclUint8, peer, c->nc, c->cs); }
  int copy_local(void *d, const void *s, size_t n) {
    return hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, c->cs) == hipSuccess ? 0 : -1;
  }
};

afs_status nccl_fail(afs_ctx *c, int r, const char *what) {
  const char *msg = r < 0 ? "HIP copy failed" : rccl().GetErrorString((ncclResult_t)r);
  return afs::fail(c, AFS_ERR_HIP, "%s: %s", what, msg);
}

afs_status comm_setup(afs_comm *m) {
  afs_ctx *c = m->ctx;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  HIP_TRY(c, hipStreamCreateWithFlags(&m->cs, hipStreamNonBlocking));
  HIP_TRY(c, hipEventCreateWithFlags(&m->ready, hipEventDisableTiming));
  HIP_TRY(c, hipEventCreateWithFlags(&m->done, hipEventDisableTiming));
  return AFS_OK;
}

// The gather in two parts, so that a caller driving several communicators in one RCCL group
// can run every fallible HIP step before the group opens: gather_prepare makes the comm's
// stream wait for the work queued so far on the context's stream; gather_post queues only the
// RCCL sends / receives (and rank 0's local copy).
// the next timing event of the pool, recorded on the comm stream
afs_status timing_event(afs_comm *m, hipEvent_t *out) {
  afs_ctx *c = m->ctx;
  if (m->tev_used == m->tev.size()) {
    hipEvent_t e = nullptr;
    HIP_TRY(c, hipEventCreate(&e));
    m->tev.push_back(e);
  }
  *out = m->tev[m->tev_used++];
  HIP_TRY(c, hipEventRecord(*out, m->cs));
  return AFS_OK;
}

afs_status gather_prepare(afs_comm *m) {
  afs_ctx *c = m->ctx;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  HIP_TRY(c, hipEventRecord(m->ready, c->stream));
  HIP_TRY(c, hipStreamWaitEvent(m->cs, m->ready, 0));
  return timing_event(m, &m->t_open);  // (after the wait: the gather's own time, not its queueing)
}

afs_status gather_post(afs_comm *m, const int16_t *local, int64_t count, int16_t *root_out,
                       const std::vector<size_t> &root_bytes) {
  RcclTransport t{m};
  const int e = afs::gather_to_root(t, local, (size_t)count * sizeof(int16_t), root_out,
                                    root_bytes.empty() ? nullptr : root_bytes.data());
  if (e) return nccl_fail(m->ctx, e, "afs_gather_pcm");
  return AFS_OK;
}

std::vector<size_t> root_bytes_of(const afs_comm *m, const int64_t *root_counts) {
  std::vector<size_t> rb;
  if (m->rank == 0 && root_counts) {
    rb.resize((size_t)m->world);
    for (int r = 0; r < m->world; ++r) rb[(size_t)r] = (size_t)root_counts[r] * sizeof(int16_t);
  }
  return rb;
}

// The HIP device that owns p (-1: host memory or unknown).
int device_of(const void *p) {
  if (!p) return -1;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged) ? at.device : -1;
}

// After a failed group: abort the RCCL communicator (its kernels stop) and mark the comm so that
// afs_comm_destroy does not wait on its stream.
void comm_abort(afs_comm *m) {
  if (!m || !m->nc) return;
  (void)hipSetDevice(m->ctx->cfg.device);
  if (rccl().CommAbort) (void)rccl().CommAbort(m->nc);
  m->nc = nullptr;
  m->aborted = true;
}

afs_status gather_finish(afs_comm *m) {
  afs_ctx *c = m->ctx;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  hipEvent_t t_close = nullptr;
  afs_status s = timing_event(m, &t_close);
  if (s != AFS_OK) return s;
  (void)t_close;  // (pairs are read in order: tev[2i], tev[2i + 1])
  HIP_TRY(c, hipEventRecord(m->done, m->cs));
  m->pending = true;
  return AFS_OK;
}

// Sum the finished gathers' event pairs into gather_ms (the comm stream has drained).
afs_status read_gather_times(afs_comm *m) {
  afs_ctx *c = m->ctx;
  for (size_t i = 0; i + 1 < m->tev_used; i += 2) {
    float x = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&x, m->tev[i], m->tev[i + 1]));
    m->gather_ms += x;
    ++m->gathers;
  }
  m->tev_used = 0;
  return AFS_OK;
}

}  // namespace

extern "C" {

void afs_shard_range(int64_t total, int32_t world, int32_t rank, int64_t *first, int64_t *count) {
  int64_t f = 0, n = 0;
  if (total > 0 && world > 0 && rank >= 0 && rank < world) afs::shard_range(total, world, rank, &f, &n);
  if (first) *first = f;
  if (count) *count = n;
}

afs_status afs_comm_unique_id(uint8_t id[AFS_COMM_ID_BYTES]) {
  if (!id) return AFS_ERR_INVALID_ARGUMENT;
  if (!rccl().ok) return AFS_ERR_UNSUPPORTED;
  ncclUniqueId u;
  if (rccl().GetUniqueId(&u) != ncclSuccess) return AFS_ERR_HIP;
  static_assert(sizeof(u.internal) == AFS_COMM_ID_BYTES, "unique id size");
  std::memcpy(id, u.internal, AFS_COMM_ID_BYTES);
  return AFS_OK;
}

afs_status afs_comm_create(afs_ctx *ctx, const uint8_t id[AFS_COMM_ID_BYTES], int32_t rank, int32_t world,
                           afs_comm **out) {
  if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world) return AFS_ERR_INVALID_ARGUMENT;
  *out = nullptr;
  if (!rccl().ok) return afs::fail(ctx, AFS_ERR_UNSUPPORTED, "%s", rccl().why.c_str());
  afs_comm *m = new afs_comm();
  m->ctx = ctx;
  m->rank = rank;
  m->world = world;
  afs_status s = comm_setup(m);
  if (s == AFS_OK) {
    ncclUniqueId u;
    std::memcpy(u.internal, id, AFS_COMM_ID_BYTES);
    const ncclResult_t r = rccl().CommInitRank(&m->nc, world, u, rank);
    if (r != ncclSuccess) s = nccl_fail(ctx, (int)r, "ncclCommInitRank");
  }
  if (s != AFS_OK) {
    afs_comm_destroy(m);
    return s;
  }
  *out = m;
  return AFS_OK;
}

afs_status afs_comm_create_all(afs_ctx *const *ctxs, int32_t n, afs_comm **comms) {
  if (!ctxs || !comms || n < 1) return AFS_ERR_INVALID_ARGUMENT;
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]) return AFS_ERR_INVALID_ARGUMENT;
    comms[i] = nullptr;
  }
  if (!rccl().ok) return afs::fail(ctxs[0], AFS_ERR_UNSUPPORTED, "%s", rccl().why.c_str());
  std::vector<int> dev((size_t)n);
  std::vector<ncclComm_t> nc((size_t)n, nullptr);
  for (int i = 0; i < n; ++i) dev[(size_t)i] = ctxs[i]->cfg.device;
  const ncclResult_t r = rccl().CommInitAll(nc.data(), n, dev.data());
  if (r != ncclSuccess) return nccl_fail(ctxs[0], (int)r, "ncclCommInitAll");
  afs_status s = AFS_OK;
  for (int i = 0; i < n; ++i) {
    afs_comm *m = new afs_comm();
    m->ctx = ctxs[i];
    m->nc = nc[(size_t)i];
    m->rank = i;
    m->world = n;
    comms[i] = m;
    if (s == AFS_OK) s = comm_setup(m);
  }
  if (s != AFS_OK)
    for (int i = 0; i < n; ++i) {
      afs_comm_destroy(comms[i]);
      comms[i] = nullptr;
    }
  return s;
}

void afs_comm_destroy(afs_comm *m) {
  if (!m) return;
  (void)hipSetDevice(m->ctx->cfg.device);
  if (m->cs && !m->aborted) (void)hipStreamSynchronize(m->cs);
  if (m->nc) (void)rccl().CommDestroy(m->nc);
  for (hipEvent_t e : m->tev) (void)hipEventDestroy(e);
  if (m->ready) (void)hipEventDestroy(m->ready);
  if (m->done) (void)hipEventDestroy(m->done);
  if (m->cs) (void)hipStreamDestroy(m->cs);
  delete m;
}

afs_status afs_gather_pcm(afs_comm *m, const int16_t *local, int64_t count, int16_t *root_out,
                          const int64_t *root_counts) {
  if (!m || count < 0 || (count > 0 && !local) || (m->rank == 0 && !root_out)) return AFS_ERR_INVALID_ARGUMENT;
  if (m->aborted) return afs::fail(m->ctx, AFS_ERR_HIP, "afs_gather_pcm: the communicator was aborted");
  // rank 0 receives into device memory of its own GPU (a buffer of another device would be a
  // fault or a silent peer write)
  if (m->rank == 0 && device_of(root_out) != m->ctx->cfg.device)
    return afs::fail(m->ctx, AFS_ERR_INVALID_ARGUMENT, "afs_gather_pcm: root_out is not device memory of device %d",
                     m->ctx->cfg.device);
  afs_status s = gather_prepare(m);
  if (s == AFS_OK) s = gather_post(m, local, count, root_out, root_bytes_of(m, root_counts));
  return s == AFS_OK ? gather_finish(m) : s;
}

afs_status afs_comm_fence(afs_comm *m) {
  if (!m) return AFS_ERR_INVALID_ARGUMENT;
  // (an aborted communicator's stream may never drain: do not make the context's stream wait on it)
  if (m->aborted) return afs::fail(m->ctx, AFS_ERR_HIP, "afs_comm_fence: the communicator was aborted");
  if (!m->pending) return AFS_OK;
  afs_ctx *c = m->ctx;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  HIP_TRY(c, hipStreamWaitEvent(c->stream, m->done, 0));
  return AFS_OK;
}

afs_status afs_comm_synchronize(afs_comm *m) {
  if (!m) return AFS_ERR_INVALID_ARGUMENT;
  if (m->aborted) return afs::fail(m->ctx, AFS_ERR_HIP, "afs_comm_synchronize: the communicator was aborted");
  afs_ctx *c = m->ctx;
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  HIP_TRY(c, hipStreamSynchronize(m->cs));
  m->pending = false;
  return read_gather_times(m);
}

afs_status afs_comm_gather_times(afs_comm *m, double *ms, int32_t *count) {
  if (!m) return AFS_ERR_INVALID_ARGUMENT;
  afs_status s = afs_comm_synchronize(m);
  if (s != AFS_OK) return s;
  if (ms) *ms = m->gather_ms;
  if (count) *count = m->gathers;
  m->gather_ms = 0.0;
  m->gathers = 0;
  return AFS_OK;
}

afs_status afs_multi_synthesize(afs_ctx *const *ctxs, afs_comm *const *comms, int32_t n, const afs_frame *frames,
                                const uint32_t *seeds, int32_t B, int32_t F, int32_t hop, int16_t *pcm_out,
                                uint8_t *nonfinite, afs_report *rep) {
  if (!ctxs || !comms || n < 1 || !ctxs[0]) return AFS_ERR_INVALID_ARGUMENT;
  afs_ctx *c0 = ctxs[0];
  if (!frames || !pcm_out || B <= 0 || F < 2 || hop < 1)
    return afs::fail(c0, AFS_ERR_INVALID_ARGUMENT, "afs_multi_synthesize: need frames, pcm_out, batch>0, num_frames>=2, hop>=1");
  for (int i = 0; i < n; ++i)
    if (!ctxs[i] || !comms[i] || comms[i]->ctx != ctxs[i] || comms[i]->rank != i || comms[i]->world != n)
      return afs::fail(c0, AFS_ERR_INVALID_ARGUMENT, "afs_multi_synthesize: comms[i] must be rank i of n on ctxs[i]");
  for (int i = 0; i < n; ++i)
    if (comms[i]->aborted) return afs::fail(c0, AFS_ERR_HIP, "afs_multi_synthesize: communicator %d was aborted", i);
  if (afs::is_device_ptr(frames) || (seeds && afs::is_device_ptr(seeds)) || (nonfinite && afs::is_device_ptr(nonfinite)))
    return afs::fail(c0, AFS_ERR_INVALID_ARGUMENT, "afs_multi_synthesize: frames, seeds and nonfinite are host arrays");
  const int64_t T = (int64_t)(F - 1) * hop;
  std::vector<uint32_t> gseeds;
  if (!seeds) {  // the global index keeps the audio independent of the device count
    gseeds.resize((size_t)B);
    for (int32_t u = 0; u < B; ++u) gseeds[(size_t)u] = (uint32_t)u + 1u;
    seeds = gseeds.data();
  }
  afs_status s;
  // one kernel width for every shard, chosen for the whole batch: the two widths agree within the
  // parity tolerances but not bit for bit, so a width chosen per shard would make the audio depend
  // on the GPU count
  const int lanes = c0->cfg.solver == AFS_SOLVER_TREE ? afs::lanes_for(c0, B) : 0;
  std::vector<int64_t> first((size_t)n), cnt((size_t)n);
  for (int i = 0; i < n; ++i) {
    afs_ctx *c = ctxs[i];
    afs::shard_range(B, n, i, &first[(size_t)i], &cnt[(size_t)i]);
    const int64_t b = cnt[(size_t)i];
    HIP_TRY(c, hipSetDevice(c->cfg.device));
    HIP_TRY(c, hipEventRecord(c->ev0, c->stream));
    if (b == 0) continue;
    if ((s = afs::ensure(c, &c->m_out, &c->m_out_bytes, (size_t)(b * T) * sizeof(double))) != AFS_OK) return s;
    if ((s = afs::ensure(c, &c->m_pcm, &c->m_pcm_bytes, (size_t)(b * T) * sizeof(int16_t))) != AFS_OK) return s;
    if ((s = afs::ensure(c, &c->m_nf, &c->m_nf_bytes, (size_t)b)) != AFS_OK) return s;
    // (queued on this device's stream; the host moves on to the next device)
    if ((s = afs::synthesize_async(c, frames + first[(size_t)i] * F, seeds + first[(size_t)i], (int32_t)b, F, hop,
                                   (double *)c->m_out, (uint8_t *)c->m_nf, lanes)) != AFS_OK)
      return s;
    HIP_TRY(c, afs::launch_to_int16((const double *)c->m_out, (int16_t *)c->m_pcm, b * T, c->stream));
  }
  for (int i = 0; i < n; ++i) HIP_TRY(ctxs[i], hipEventRecord(ctxs[i]->ev1, ctxs[i]->stream));
  int16_t *root = pcm_out;
  const int out_dev = device_of(pcm_out);
  const bool host_out = out_dev < 0;
  if (!host_out && out_dev != c0->cfg.device)
    return afs::fail(c0, AFS_ERR_INVALID_ARGUMENT, "afs_multi_synthesize: pcm_out is device memory of device %d, not of "
                     "ctxs[0]'s device %d", out_dev, c0->cfg.device);
  if (host_out) {
    HIP_TRY(c0, hipSetDevice(c0->cfg.device));
    if ((s = afs::ensure(c0, &c0->m_root, &c0->m_root_bytes, (size_t)B * (size_t)T * sizeof(int16_t))) != AFS_OK)
      return s;
    root = (int16_t *)c0->m_root;
  }
  std::vector<int64_t> counts((size_t)n);
  for (int i = 0; i < n; ++i) counts[(size_t)i] = cnt[(size_t)i] * T;
  // every rank's sends / receives in one group (one host thread drives all communicators); the
  // HIP steps that can fail (events, stream waits) all run before the group opens, so a failure
  // never leaves a receive without its send
  for (int i = 0; i < n; ++i)
    if ((s = gather_prepare(comms[i])) != AFS_OK) return s;
  const std::vector<size_t> rb0 = root_bytes_of(comms[0], counts.data());
  if (rccl().GroupStart() != ncclSuccess) return afs::fail(c0, AFS_ERR_HIP, "ncclGroupStart failed");
  afs_status gs = AFS_OK;
  for (int i = 0; i < n && gs == AFS_OK; ++i)
    gs = gather_post(comms[i], (const int16_t *)ctxs[i]->m_pcm, counts[(size_t)i], i == 0 ? root : nullptr,
                     i == 0 ? rb0 : std::vector<size_t>());
  const ncclResult_t ge = rccl().GroupEnd();
  if (gs != AFS_OK || ge != ncclSuccess) {
    // an incomplete group can leave a receive without its send: abort the communicators
    // (afs_comm_destroy then skips the stream wait that would block on it)
    for (int i = 0; i < n; ++i) comm_abort(comms[i]);
    return gs != AFS_OK ? gs : nccl_fail(c0, (int)ge, "ncclGroupEnd");
  }
  for (int i = 0; i < n; ++i)
    if ((s = gather_finish(comms[i])) != AFS_OK) return s;
  HIP_TRY(c0, hipSetDevice(c0->cfg.device));
  if (host_out) {
    HIP_TRY(c0, hipStreamWaitEvent(c0->stream, comms[0]->done, 0));
    HIP_TRY(c0, hipMemcpyAsync(pcm_out, root, (size_t)B * (size_t)T * sizeof(int16_t), hipMemcpyDeviceToHost, c0->stream));
  }
  double ms = 0.0;
  int32_t nonfin = 0;
  std::vector<uint8_t> flags_local;
  if (!nonfinite) {
    flags_local.assign((size_t)B, 0);
    nonfinite = flags_local.data();
  }
  for (int i = 0; i < n; ++i) {
    afs_ctx *c = ctxs[i];
    HIP_TRY(c, hipSetDevice(c->cfg.device));
    if (cnt[(size_t)i] > 0)
      HIP_TRY(c, hipMemcpyAsync(nonfinite + first[(size_t)i], c->m_nf, (size_t)cnt[(size_t)i], hipMemcpyDeviceToHost,
                                c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if ((s = afs_comm_synchronize(comms[i])) != AFS_OK) return s;
    float x = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&x, c->ev0, c->ev1));
    ms = std::max(ms, (double)x);
  }
  for (int32_t u = 0; u < B; ++u) nonfin += nonfinite[u] ? 1 : 0;
  if (rep) {
    std::memset(rep, 0, sizeof *rep);
    rep->device_ms = ms;
    rep->samples = (int64_t)B * T;
    rep->nonfinite_utterances = nonfin;
    rep->kernel = c0->cfg.solver;
  }
  return AFS_OK;
}

}  // extern "C"
