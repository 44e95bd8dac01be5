// picp_comm.cpp -- the multi-GPU batch split's communicator: RCCL driven from the C++ host.
//
// independent frames are sharded over the GPUs of one node, one process per GPU,
// with no data-path collective; the only exchange is one all-gather of the per-frame results
// (pose + stats, 128 B per frame) at the end, plus the max-over-ranks of a timing and a barrier.
// Each rank owns one picp_comm bound to its device; the RCCL unique id travels over whatever
// out-of-band channel the launcher has (bench.py: the gloo store, bytes only).
//
// librccl is opened with dlopen on the first picp_comm_* call, so single-GPU users of
// libpicp_amd.so never load it.  RCCL routes the all-gather over xGMI between the node's GPUs.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <mutex>

#include "picp_c.h"
#include "picp_comm.h"
#include "picp_host.h"

namespace {

struct RcclApi {
  void* so = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
  char why[256] = {0};
};

RcclApi g_rccl;
std::once_flag g_rccl_once;

template <typename F>
bool sym(void* so, const char* name, F* out) {
  *out = reinterpret_cast<F>(dlsym(so, name));
  return *out != nullptr;
}

const RcclApi& rccl() {
  std::call_once(g_rccl_once, [] {
    RcclApi& a = g_rccl;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names)
      if ((a.so = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!a.so) {
      snprintf(a.why, sizeof(a.why), "dlopen(librccl.so.1): %s", dlerror());
      return;
    }
    a.ok = sym(a.so, "ncclGetUniqueId", &a.get_unique_id) && sym(a.so, "ncclCommInitRank", &a.comm_init_rank) &&
           sym(a.so, "ncclCommDestroy", &a.comm_destroy) && sym(a.so, "ncclAllGather", &a.all_gather) &&
           sym(a.so, "ncclAllReduce", &a.all_reduce) && sym(a.so, "ncclGetErrorString", &a.error_string);
    if (!a.ok) snprintf(a.why, sizeof(a.why), "librccl lacks a required symbol");
  });
  return g_rccl;
}

#define RCCL_API_OR_FAIL()                                                              \
  const RcclApi& R = rccl();                                                            \
  if (!R.ok) return picp_set_err(PICP_ERR_DEVICE, "RCCL unavailable: %s", R.why)

#define NCCL_TRY(expr)                                                                  \
  do {                                                                                  \
    ncclResult_t r_ = (expr);                                                           \
    if (r_ != ncclSuccess)                                                              \
      return picp_set_err(PICP_ERR_DEVICE, "%s failed: %s", #expr, R.error_string(r_)); \
  } while (0)

}  // namespace

struct picp_comm {
  int device = 0, world = 1, rank = 0;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;   // the communicator's own stream (timing reductions, barrier)
  double* red_d = nullptr;        // reduction scratch
  int red_cap = 0;
  void* send_d = nullptr;         // all-gather staging (grown on demand)
  size_t send_cap = 0;
  void* recv_d = nullptr;
  size_t recv_cap = 0;
};

extern "C" int picp_shard_range(int64_t n_items, int world, int rank, int64_t* first, int64_t* last) {
  CHECK_ARG(first && last, "picp_shard_range: null output");
  CHECK_ARG(n_items >= 0 && world >= 1 && rank >= 0 && rank < world, "picp_shard_range: bad world/rank");
  const int64_t base = n_items / world, extra = n_items % world;
  *first = rank * base + std::min<int64_t>(rank, extra);
  *last = *first + base + (rank < extra ? 1 : 0);
  return PICP_OK;
}

extern "C" int64_t picp_shard_pad(int64_t n_items, int world) {
  if (n_items < 0 || world < 1) return -1;
  return (n_items + world - 1) / world;
}

extern "C" int picp_shard_unpack(int64_t n_items, int world, int64_t item_bytes, const void* padded, void* out) {
  CHECK_ARG(n_items >= 0 && world >= 1 && item_bytes >= 1, "picp_shard_unpack: bad size");
  CHECK_ARG(n_items == 0 || (padded && out), "picp_shard_unpack: null buffer");
  const int64_t pad = picp_shard_pad(n_items, world);
  const char* src = (const char*)padded;
  char* dst = (char*)out;
  for (int r = 0; r < world; ++r) {
    int64_t a = 0, e = 0;
    picp_shard_range(n_items, world, r, &a, &e);
    if (e > a) memcpy(dst + a * item_bytes, src + (size_t)r * pad * item_bytes, (size_t)(e - a) * item_bytes);
  }
  return PICP_OK;
}

extern "C" int picp_comm_unique_id(uint8_t id[PICP_COMM_ID_BYTES]) {
  CHECK_ARG(id, "picp_comm_unique_id: null output");
  static_assert(sizeof(ncclUniqueId) == PICP_COMM_ID_BYTES, "RCCL unique id size");
  RCCL_API_OR_FAIL();
  ncclUniqueId u;
  NCCL_TRY(R.get_unique_id(&u));
  memcpy(id, &u, sizeof(u));
  return PICP_OK;
}

extern "C" int picp_comm_create(picp_comm_t** out, int device, int world, int rank,
                                const uint8_t id[PICP_COMM_ID_BYTES]) {
  CHECK_ARG(out && id, "picp_comm_create: null argument");
  CHECK_ARG(world >= 1 && rank >= 0 && rank < world, "picp_comm_create: bad world/rank");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  CHECK_ARG(device >= 0 && device < ndev, "picp_comm_create: no such HIP device");
  RCCL_API_OR_FAIL();
  HIP_TRY(hipSetDevice(device));
  picp_comm* c = new picp_comm();
  c->device = device;
  c->world = world;
  c->rank = rank;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->red_d, 64 * sizeof(double));
  if (e != hipSuccess) {
    picp_comm_destroy(c);
    return picp_set_err(PICP_ERR_DEVICE, "picp_comm_create: %s", hipGetErrorString(e));
  }
  c->red_cap = 64;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  const ncclResult_t r = R.comm_init_rank(&c->comm, world, u, rank);  // blocks until all ranks join
  if (r != ncclSuccess) {
    c->comm = nullptr;
    picp_comm_destroy(c);
    return picp_set_err(PICP_ERR_DEVICE, "ncclCommInitRank(world %d, rank %d): %s", world, rank, R.error_string(r));
  }
  *out = c;
  return PICP_OK;
}

extern "C" int picp_comm_destroy(picp_comm_t* c) {
  if (!c) return PICP_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->comm && g_rccl.ok) g_rccl.comm_destroy(c->comm);
  if (c->red_d) hipFree(c->red_d);
  if (c->send_d) hipFree(c->send_d);
  if (c->recv_d) hipFree(c->recv_d);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return PICP_OK;
}

extern "C" int picp_comm_info(picp_comm_t* c, int* device, int* world, int* rank) {
  CHECK_ARG(c, "picp_comm_info: null communicator");
  if (device) *device = c->device;
  if (world) *world = c->world;
  if (rank) *rank = c->rank;
  return PICP_OK;
}

extern "C" int picp_comm_allreduce_max(picp_comm_t* c, double* values, int n) {
  CHECK_ARG(c && values && n >= 1 && n <= 64, "picp_comm_allreduce_max: bad argument (1..64 values)");
  RCCL_API_OR_FAIL();
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(c->red_d, values, (size_t)n * sizeof(double), hipMemcpyHostToDevice, c->stream));
  NCCL_TRY(R.all_reduce(c->red_d, c->red_d, (size_t)n, ncclFloat64, ncclMax, c->comm, c->stream));
  HIP_TRY(hipMemcpyAsync(values, c->red_d, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PICP_OK;
}

extern "C" int picp_comm_barrier(picp_comm_t* c) {
  double one = 1.0;
  return picp_comm_allreduce_max(c, &one, 1);
}

// All-gather `bytes` per rank from device memory `send` into the communicator's receive buffer
// (world x bytes, rank order), enqueued on `stream` after whatever the stream already holds.
// *recv receives the device pointer.  The caller synchronizes the stream before reading it.
int picp_comm_allgather_dev(picp_comm* c, const void* send, size_t bytes, hipStream_t stream, const void** recv) {
  RCCL_API_OR_FAIL();
  HIP_TRY(hipSetDevice(c->device));
  const size_t total = bytes * (size_t)c->world;
  if (bytes > c->send_cap) {
    if (c->send_d) hipFree(c->send_d);
    c->send_d = nullptr;
    c->send_cap = 0;
    HIP_TRY(hipMalloc(&c->send_d, bytes));
    c->send_cap = bytes;
  }
  if (total > c->recv_cap) {
    if (c->recv_d) hipFree(c->recv_d);
    c->recv_d = nullptr;
    c->recv_cap = 0;
    HIP_TRY(hipMalloc(&c->recv_d, total));
    c->recv_cap = total;
  }
  if (send != c->send_d && bytes)
    HIP_TRY(hipMemcpyAsync(c->send_d, send, bytes, hipMemcpyDeviceToDevice, stream));
  NCCL_TRY(R.all_gather(c->send_d, c->recv_d, bytes, ncclUint8, c->comm, stream));
  *recv = c->recv_d;
  return PICP_OK;
}

int picp_comm_device(const picp_comm* c) { return c->device; }
int picp_comm_world(const picp_comm* c) { return c->world; }
int picp_comm_rank(const picp_comm* c) { return c->rank; }
void* picp_comm_send_buffer(picp_comm* c, size_t bytes) {
  if (bytes > c->send_cap) {
    if (c->send_d) hipFree(c->send_d);
    c->send_d = nullptr;
    c->send_cap = 0;
    if (hipMalloc(&c->send_d, bytes) != hipSuccess) return nullptr;
    c->send_cap = bytes;
  }
  return c->send_d;
}
