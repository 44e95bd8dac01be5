// picp_comm.h -- runtime-internal view of the RCCL communicator (picp_comm.cpp) for the batch
// all-gather in picp_runtime.cpp.  Not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

struct picp_comm;

// device staging buffer of at least `bytes` for the all-gather send side (nullptr on OOM)
__attribute__((visibility("hidden"))) void* picp_comm_send_buffer(picp_comm* c, size_t bytes);
// all-gather `bytes` per rank from device memory `send`, enqueued on `stream`; *recv = the
// device receive buffer (world x bytes, rank order), valid once the stream is synchronized
__attribute__((visibility("hidden"))) int picp_comm_allgather_dev(picp_comm* c, const void* send, size_t bytes,
                                                                  hipStream_t stream, const void** recv);
__attribute__((visibility("hidden"))) int picp_comm_device(const picp_comm* c);
__attribute__((visibility("hidden"))) int picp_comm_world(const picp_comm* c);
__attribute__((visibility("hidden"))) int picp_comm_rank(const picp_comm* c);
