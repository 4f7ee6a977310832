// Native bucketed gradient reducer (include/liteasr_comm.h): one HIP stream of its own, one
// ready event per bucket, in-place ncclAllReduce(ncclAvg) over contiguous slices of the flat
// fp32 gradient buffer.  Mirrors liteasr_amd/distributed/ddp.py:FlatReducer's bucket order
// and finalize semantics (which restate torch DDP as used at liteasr/trainer.py:76-88).
#include "../../../include/liteasr_comm.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(x)                                                                     \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return fail(-2, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

#define NCCL_TRY(x)                                                                          \
  do {                                                                                       \
    ncclResult_t e_ = (x);                                                                   \
    if (e_ != ncclSuccess) return fail(-3, std::string(#x ": ") + ncclGetErrorString(e_));    \
  } while (0)

}  // namespace

struct lasr_reducer {
  ncclComm_t comm = nullptr;
  bool owns_comm = false;
  int device = 0;
  int world = 1;
  // world 1: the average over one rank is the identity, so no collective, no stream wait and
  // no event is issued (what the torch.distributed path does at world 1); set_single_rank_
  // collectives(1) issues them anyway (the world-1 measurement of RCCL's cost to the compute)
  bool single_rank_collectives = false;
  float* grad = nullptr;
  int64_t numel = 0;
  std::vector<int64_t> lo, hi;
  std::vector<char> marked;
  int next = 0;               // next bucket to launch (strict order)
  hipStream_t stream = nullptr;
  std::vector<hipEvent_t> ready;  // per bucket: producer-side completion
  hipEvent_t done = nullptr;      // comm-side completion of the step's collectives
};

namespace {

// Selects `device` for the scope and restores the caller's device afterwards.
struct DeviceGuard {
  int prev = -1, rc = 0;
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    rc = hipSetDevice(device) != hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int check_buckets(int64_t numel, const int64_t* lo, const int64_t* hi, int n) {
  if (n <= 0 || !lo || !hi) return fail(-1, "no buckets");
  std::vector<std::pair<int64_t, int64_t>> v;
  for (int b = 0; b < n; ++b) {
    if (lo[b] < 0 || hi[b] > numel || lo[b] >= hi[b])
      return fail(-1, "bucket " + std::to_string(b) + " outside [0, numel) or empty");
    v.emplace_back(lo[b], hi[b]);
  }
  std::sort(v.begin(), v.end());
  for (size_t i = 1; i < v.size(); ++i)
    if (v[i].first < v[i - 1].second) return fail(-1, "buckets overlap");
  return 0;
}

int setup(lasr_reducer* r, int device, float* grad, int64_t numel, const int64_t* lo,
          const int64_t* hi, int n) {
  if (!grad) return fail(-1, "null gradient buffer");
  if (int rc = check_buckets(numel, lo, hi, n)) return rc;
  r->device = device;
  r->grad = grad;
  r->lo.assign(lo, lo + n);
  r->hi.assign(hi, hi + n);
  r->numel = numel;
  r->marked.assign(n, 0);
  // the caller's current device is restored on return (the stream and events belong to
  // `device`, whatever device the training thread has selected)
  DeviceGuard dg(device);
  if (dg.rc) return fail(-2, "hipSetDevice failed");
  HIP_TRY(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
  r->ready.assign(n, nullptr);
  for (int b = 0; b < n; ++b) HIP_TRY(hipEventCreateWithFlags(&r->ready[b], hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&r->done, hipEventDisableTiming));
  return 0;
}

bool collectives(const lasr_reducer* r) { return r->world > 1 || r->single_rank_collectives; }

int launch(lasr_reducer* r, int b) {
  if (!collectives(r)) return 0;
  HIP_TRY(hipStreamWaitEvent(r->stream, r->ready[b], 0));
  float* p = r->grad + r->lo[b];
  NCCL_TRY(ncclAllReduce(p, p, (size_t)(r->hi[b] - r->lo[b]), ncclFloat32, ncclAvg, r->comm, r->stream));
  return 0;
}

void release(lasr_reducer* r) {
  DeviceGuard dg(r->device);  // the stream, events and communicator live on r->device
  if (r->stream) (void)hipStreamSynchronize(r->stream);
  for (hipEvent_t e : r->ready)
    if (e) (void)hipEventDestroy(e);
  if (r->done) (void)hipEventDestroy(r->done);
  if (r->stream) (void)hipStreamDestroy(r->stream);
  if (r->owns_comm && r->comm) ncclCommDestroy(r->comm);
  delete r;
}

}  // namespace

extern "C" {

int lasr_reducer_uid_bytes(void) { return (int)sizeof(ncclUniqueId); }

int lasr_reducer_get_unique_id(void* uid) {
  if (!uid) return fail(-1, "null uid");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  std::memcpy(uid, &id, sizeof(id));
  return 0;
}

int lasr_reducer_create(lasr_reducer** out, const void* uid, int world, int rank, int device,
                        float* grad, int64_t numel, const int64_t* bucket_lo,
                        const int64_t* bucket_hi, int n_buckets) {
  if (!out || !uid) return fail(-1, "null argument");
  if (world < 1 || rank < 0 || rank >= world) return fail(-1, "rank outside [0, world)");
  *out = nullptr;
  auto* r = new lasr_reducer;
  if (int rc = setup(r, device, grad, numel, bucket_lo, bucket_hi, n_buckets)) {
    std::string keep = g_err;
    release(r);
    return fail(rc, keep);
  }
  r->world = world;
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  ncclResult_t e = ncclCommInitRank(&r->comm, world, id, rank);
  if (e != ncclSuccess) {
    r->comm = nullptr;
    release(r);
    return fail(-3, std::string("ncclCommInitRank: ") + ncclGetErrorString(e));
  }
  r->owns_comm = true;
  *out = r;
  return 0;
}

int lasr_reducer_create_from_comm(lasr_reducer** out, void* comm, int device, float* grad,
                                  int64_t numel, const int64_t* bucket_lo,
                                  const int64_t* bucket_hi, int n_buckets) {
  if (!out || !comm) return fail(-1, "null argument");
  *out = nullptr;
  int nranks = 0;  // queried before anything is allocated: a failure leaks nothing
  NCCL_TRY(ncclCommCount((ncclComm_t)comm, &nranks));
  auto* r = new lasr_reducer;
  if (int rc = setup(r, device, grad, numel, bucket_lo, bucket_hi, n_buckets)) {
    std::string keep = g_err;
    release(r);
    return fail(rc, keep);
  }
  r->comm = (ncclComm_t)comm;
  r->world = nranks;
  *out = r;
  return 0;
}

int lasr_reducer_mark_grad_ready(lasr_reducer* r, int bucket, hipStream_t producer) {
  if (!r) return fail(-1, "null reducer");
  const int n = (int)r->lo.size();
  if (bucket < 0 || bucket >= n) return fail(-1, "bucket index out of range");
  if (r->marked[bucket]) return fail(-1, "bucket " + std::to_string(bucket) + " marked twice in one step");
  r->marked[bucket] = 1;
  if (collectives(r)) HIP_TRY(hipEventRecord(r->ready[bucket], producer));
  while (r->next < n && r->marked[r->next]) {
    if (int rc = launch(r, r->next)) return rc;
    ++r->next;
  }
  return 0;
}

int lasr_reducer_finalize(lasr_reducer* r, hipStream_t consumer) {
  if (!r) return fail(-1, "null reducer");
  const int n = (int)r->lo.size();
  for (int b = r->next; b < n; ++b) {
    if (!r->marked[b] && collectives(r)) HIP_TRY(hipEventRecord(r->ready[b], consumer));
    if (int rc = launch(r, b)) return rc;
  }
  if (collectives(r)) {
    HIP_TRY(hipEventRecord(r->done, r->stream));
    HIP_TRY(hipStreamWaitEvent(consumer, r->done, 0));
  }
  std::fill(r->marked.begin(), r->marked.end(), 0);
  r->next = 0;
  return 0;
}

int lasr_reducer_launched(const lasr_reducer* r) { return r ? r->next : -1; }

int lasr_reducer_reset(lasr_reducer* r) {
  if (!r) return fail(-1, "null reducer");
  std::fill(r->marked.begin(), r->marked.end(), 0);
  r->next = 0;
  return 0;
}

int lasr_reducer_rebind(lasr_reducer* r, float* grad, int64_t numel) {
  if (!r || !grad) return fail(-1, "null argument");
  if (numel != r->numel)
    return fail(-1, "rebind: numel " + std::to_string(numel) + " != " + std::to_string(r->numel));
  if (r->next != 0 || std::find(r->marked.begin(), r->marked.end(), 1) != r->marked.end())
    return fail(-1, "rebind inside a step (buckets already marked)");
  // the communicator, stream and events belong to r->device: a buffer on another device (a
  // device move of the model) needs a new reducer, not a rebind
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, grad) != hipSuccess) {
    (void)hipGetLastError();
    return fail(-1, "rebind: the buffer is not device memory");
  }
  if (at.type != hipMemoryTypeDevice) return fail(-1, "rebind: the buffer is not device memory");
  if (at.device != r->device)
    return fail(-1, "rebind: the buffer is on device " + std::to_string(at.device) + ", the reducer on device " +
                        std::to_string(r->device) + " (a device move needs a new reducer)");
  r->grad = grad;
  return 0;
}

int lasr_reducer_set_single_rank_collectives(lasr_reducer* r, int on) {
  if (!r) return fail(-1, "null reducer");
  if (r->next != 0 || std::find(r->marked.begin(), r->marked.end(), 1) != r->marked.end())
    return fail(-1, "set_single_rank_collectives inside a step");
  r->single_rank_collectives = on != 0;
  return 0;
}

const float* lasr_reducer_grad(const lasr_reducer* r) { return r ? r->grad : nullptr; }

int lasr_reducer_destroy(lasr_reducer* r) {
  if (!r) return 0;
  release(r);  // selects r->device, drains the stream, frees events / stream / communicator
  return 0;
}

const char* lasr_comm_last_error(void) { return g_err.c_str(); }

}  // extern "C"
