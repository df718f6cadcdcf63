// Native RCCL point-to-point transport for pipeline-stage boundaries.
//
// The boundary message is one contiguous byte buffer, so a stage hand-off is a single ncclSend /
// ncclRecv pair over xGMI.  A handle here is one *channel*: a communicator (for a pipeline edge: the
// two ranks of the edge, bootstrapped from a unique id the Python side hands over through the
// torch.distributed store) plus its own non-blocking stream.  A middle stage therefore owns two
// channels - the receive edge from its upstream and the send edge to its downstream - on two
// streams, so a receive posted ahead for the next micro-batch never sits in front of the send of the
// current one.  Ordering with the compute stream is expressed with HIP events only:
//
//   send: compute stream --event--> channel stream: ncclSend --event (per op, Python side)--> waiter
//   recv: channel stream: ncclRecv --event (per op)--> compute stream (waits before the decode kernel)
//
// so no stream ever blocks the host.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#define EDGE_API extern "C" __attribute__((visibility("default")))

constexpr int NEV = 64;  // ring of events for stream<->stream ordering (a wait captures the event's state)

struct EdgeComm {
  ncclComm_t comm;
  hipStream_t stream;
  hipEvent_t ev[NEV];
  int ev_next = 0;
  int rank, nranks;
  hipEvent_t next_event() { return ev[ev_next++ % NEV]; }
};

static int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? 0 : 1000 + (int)r; }

EDGE_API int edge_rccl_id_bytes() { return (int)sizeof(ncclUniqueId); }

EDGE_API int edge_rccl_unique_id(char* out) {
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return nccl_rc(r);
  memcpy(out, &id, sizeof(id));
  return 0;
}

EDGE_API int edge_rccl_init(void** handle, int nranks, const char* id_bytes, int rank, int device) {
  *handle = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  EdgeComm* c = new EdgeComm();
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_rc(r);
  }
  e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    ncclCommDestroy(c->comm);
    delete c;
    return (int)e;
  }
  for (int i = 0; i < NEV; ++i) {
    e = hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming);
    if (e != hipSuccess) return (int)e;
  }
  c->rank = rank;
  c->nranks = nranks;
  *handle = c;
  return 0;
}

EDGE_API int edge_rccl_destroy(void* handle) {
  EdgeComm* c = (EdgeComm*)handle;
  if (!c) return 0;
  (void)hipStreamSynchronize(c->stream);
  const ncclResult_t r = ncclCommDestroy(c->comm);
  for (int i = 0; i < NEV; ++i) (void)hipEventDestroy(c->ev[i]);
  // The comm stream is deliberately NOT destroyed: buffers handed to RCCL are tied to it through the
  // torch caching allocator (record_stream), which records events on it when those blocks are freed,
  // possibly at interpreter exit.  A stream per communicator for the process lifetime is harmless.
  delete c;
  return nccl_rc(r);
}

// Make the comm stream wait for everything queued so far on `compute` (the producer of a send buffer).
EDGE_API int edge_rccl_wait_for(void* handle, hipStream_t compute) {
  EdgeComm* c = (EdgeComm*)handle;
  hipEvent_t ev = c->next_event();
  hipError_t e = hipEventRecord(ev, compute);
  if (e != hipSuccess) return (int)e;
  return (int)hipStreamWaitEvent(c->stream, ev, 0);
}

// Make `compute` wait for everything queued so far on the comm stream (a finished receive).
EDGE_API int edge_rccl_signal_to(void* handle, hipStream_t compute) {
  EdgeComm* c = (EdgeComm*)handle;
  hipEvent_t ev = c->next_event();
  hipError_t e = hipEventRecord(ev, c->stream);
  if (e != hipSuccess) return (int)e;
  return (int)hipStreamWaitEvent(compute, ev, 0);
}

EDGE_API int edge_rccl_group_start() { return nccl_rc(ncclGroupStart()); }
EDGE_API int edge_rccl_group_end() { return nccl_rc(ncclGroupEnd()); }

EDGE_API int edge_rccl_send(void* handle, const void* buf, long long bytes, int peer) {
  EdgeComm* c = (EdgeComm*)handle;
  return nccl_rc(ncclSend(buf, (size_t)bytes, ncclUint8, peer, c->comm, c->stream));
}

EDGE_API int edge_rccl_recv(void* handle, void* buf, long long bytes, int peer) {
  EdgeComm* c = (EdgeComm*)handle;
  return nccl_rc(ncclRecv(buf, (size_t)bytes, ncclUint8, peer, c->comm, c->stream));
}

EDGE_API int edge_rccl_allreduce_sum_f64(void* handle, void* buf, long long count) {
  EdgeComm* c = (EdgeComm*)handle;
  return nccl_rc(ncclAllReduce(buf, buf, (size_t)count, ncclFloat64, ncclSum, c->comm, c->stream));
}

EDGE_API int edge_rccl_stream_sync(void* handle) {
  return (int)hipStreamSynchronize(((EdgeComm*)handle)->stream);
}

EDGE_API long long edge_rccl_stream(void* handle) { return (long long)((EdgeComm*)handle)->stream; }
