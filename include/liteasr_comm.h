/* liteasr_comm.h -- native bucketed gradient reducer of the MI355X LiteASR training path.
 *
 * Host C ABI (libliteasr_comm.so: C++17 over the HIP runtime and RCCL, no device code of its
 * own).  The flat fp32 gradient buffer of a FlatParams model is cut into contiguous buckets;
 * the backward marks a bucket ready on the stream that produced its gradients, and the
 * reducer launches that bucket's in-place ncclAllReduce(ncclAvg) on its own HIP stream, in
 * bucket order (every rank issues the same collective sequence), so communication overlaps
 * the rest of the backward.  finalize() launches buckets that never fired and makes the
 * consumer (optimizer) stream wait for every collective.
 *
 * Replaces (reference, Python over torch DDP):
 *   liteasr/trainer.py:76-88    DistributedDataParallel(model, device_ids=[rank]) -- the
 *                               gradient bucketing + all-reduce (average) it performs
 *   liteasr/trainer.py:142-147  model.no_sync() during gradient accumulation (the caller
 *                               simply does not mark buckets)
 *   SURVEY.md §8(b)             "the comm side exports lasr_reducer_*"
 *
 * Conventions: 0 = success, negative = error (message in lasr_comm_last_error(), thread-
 * local).  The caller owns the gradient buffer; the reducer owns its stream, events and --
 * when created from a unique id -- its RCCL communicator.  Not thread-safe (one reducer per
 * process / device, driven from the training thread), stream-ordered, no host sync.
 */
#ifndef LITEASR_COMM_H
#define LITEASR_COMM_H

#include <stdint.h>

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lasr_reducer lasr_reducer;

/* size in bytes of an RCCL unique id (rank 0 creates it, every rank passes the same bytes) */
int lasr_reducer_uid_bytes(void);

/* rank 0: fill `uid` (lasr_reducer_uid_bytes() bytes) with a fresh communicator id */
int lasr_reducer_get_unique_id(void* uid);

/* Create a reducer with its own communicator (ncclCommInitRank on `device`).
 * Bucket b covers grad[bucket_lo[b], bucket_hi[b]) (fp32 elements); buckets must be
 * non-empty, inside [0, numel) and pairwise disjoint. */
int lasr_reducer_create(lasr_reducer** out, const void* uid, int world, int rank, int device,
                        float* grad, int64_t numel, const int64_t* bucket_lo,
                        const int64_t* bucket_hi, int n_buckets);

/* Same over an existing communicator (an ncclComm_t passed as void*; the caller keeps it). */
int lasr_reducer_create_from_comm(lasr_reducer** out, void* comm, int device, float* grad,
                                  int64_t numel, const int64_t* bucket_lo,
                                  const int64_t* bucket_hi, int n_buckets);

/* Bucket `bucket`'s gradients are complete on `producer`.  Launches, in order, every bucket
 * from the next unlaunched one on that is marked.  Marking a bucket twice in one step is an
 * error. */
int lasr_reducer_mark_grad_ready(lasr_reducer* r, int bucket, hipStream_t producer);

/* End of the step: launch the buckets never marked (their gradients are complete on
 * `consumer`), make `consumer` wait for every collective, reset for the next step. */
int lasr_reducer_finalize(lasr_reducer* r, hipStream_t consumer);

/* number of buckets launched so far in the current step */
int lasr_reducer_launched(const lasr_reducer* r);

/* Abandon the current step's bookkeeping (marked flags, next bucket) without launching
 * anything: after a backward that stopped part-way (an exception, an abandoned capture).
 * Collectives already launched stay in flight on the reducer's stream. */
int lasr_reducer_reset(lasr_reducer* r);

/* Point the reducer at a new gradient buffer of the same numel and the same device (the caller
 * reallocated it).  Only between steps.  A buffer on another device is refused: the
 * communicator, stream and events belong to the creation device, so a device move of the
 * model needs a new reducer. */
int lasr_reducer_rebind(lasr_reducer* r, float* grad, int64_t numel);

/* At world 1 the average is the identity and the reducer issues nothing (no event, no
 * collective), as the torch.distributed path does.  on != 0 issues the 1-rank collectives
 * anyway: the world-1 measurement of what RCCL's kernels cost the overlapped backward.
 * Only between steps; no effect at world > 1. */
int lasr_reducer_set_single_rank_collectives(lasr_reducer* r, int on);

/* the gradient buffer the reducer currently averages */
const float* lasr_reducer_grad(const lasr_reducer* r);

/* drains the reducer's stream (on its device), then frees it and, if owned, the communicator */
int lasr_reducer_destroy(lasr_reducer* r);

const char* lasr_comm_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* LITEASR_COMM_H */
