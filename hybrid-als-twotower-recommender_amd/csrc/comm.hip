// The multi-GPU exchange steps of the hot path for hosts that do not use
// torch.distributed (SURVEY §8(b) proposal, §8(e)): one process per GPU,
// RCCL over xGMI.
//   C1 hrec_allgather: the replicated factor matrix after each ALS
//      half-sweep (what src/als_engine.py does with all_gather_into_tensor);
//   C2 hrec_allreduce_minmax: the global per-user min / max of each model's
//      score row across item shards (src/recommend.py global_minmax: one
//      MIN all-reduce over [min | -max]);
//   C3 = hrec_allgather of the per-shard top-k candidates.
// RCCL is bound at hrec_comm_init by dlopen: the copy a process already has
// loaded (PyTorch's) is used when there is one, so one process never holds
// two RCCL builds; otherwise librccl.so.1 from the loader path or /opt/rocm.
#include <dlfcn.h>
#include <string.h>

#include <mutex>

#include "common.h"

namespace hrec {

// The few RCCL entry points used (rccl.h types restated: opaque id of 128
// bytes, enums as int; the ABI of ncclGetUniqueId / ncclCommInitRank /
// ncclAllGather / ncclAllReduce / ncclCommDestroy / ncclGetErrorString).
struct RcclId {
  char internal[128];
};
typedef int (*rccl_get_id_t)(RcclId*);
typedef int (*rccl_init_t)(void**, int, RcclId, int);
typedef int (*rccl_allgather_t)(const void*, void*, size_t, int, void*, hipStream_t);
typedef int (*rccl_allreduce_t)(const void*, void*, size_t, int, int, void*, hipStream_t);
typedef int (*rccl_destroy_t)(void*);
typedef const char* (*rccl_err_t)(int);

struct Rccl {
  void* handle = nullptr;
  rccl_get_id_t get_id = nullptr;
  rccl_init_t init = nullptr;
  rccl_allgather_t allgather = nullptr;
  rccl_allreduce_t allreduce = nullptr;
  rccl_destroy_t destroy = nullptr;
  rccl_err_t err = nullptr;
};

static const Rccl* rccl() {
  static std::once_flag once;
  static Rccl r;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    Rccl t;
    t.handle = h;
    t.get_id = (rccl_get_id_t)dlsym(h, "ncclGetUniqueId");
    t.init = (rccl_init_t)dlsym(h, "ncclCommInitRank");
    t.allgather = (rccl_allgather_t)dlsym(h, "ncclAllGather");
    t.allreduce = (rccl_allreduce_t)dlsym(h, "ncclAllReduce");
    t.destroy = (rccl_destroy_t)dlsym(h, "ncclCommDestroy");
    t.err = (rccl_err_t)dlsym(h, "ncclGetErrorString");
    if (t.get_id && t.init && t.allgather && t.allreduce && t.destroy) r = t;
  });
  return r.handle && r.init ? &r : nullptr;
}

struct Comm {
  void* nccl;
  int rank, world;
};

static int rccl_fail(const Rccl* r, int rc, const char* what) {
  set_error("%s: RCCL error %d (%s)", what, rc, r->err ? r->err(rc) : "?");
  return HREC_E_LAUNCH;
}

// mm[0 .. n) *= -1 (the max rows travel negated through the MIN all-reduce)
__global__ __launch_bounds__(256) void negate_f32_kernel(float* __restrict__ x, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) x[i] = -x[i];
}

static int negate_rows(float* x, int64_t n, hipStream_t s) {
  int64_t g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(negate_f32_kernel, dim3((unsigned)g), dim3(256), 0, s, x, n);
  return check_launch("negate_f32_kernel");
}

}  // namespace hrec

using namespace hrec;

extern "C" int hrec_comm_get_unique_id(uint8_t* id_out) {
  HREC_REQUIRE(id_out, "comm_get_unique_id: null output");
  const Rccl* r = rccl();
  if (!r) {
    set_error("comm_get_unique_id: librccl.so.1 could not be loaded");
    return HREC_E_UNSUPPORTED;
  }
  RcclId id;
  const int rc = r->get_id(&id);
  if (rc) return rccl_fail(r, rc, "comm_get_unique_id");
  memcpy(id_out, id.internal, sizeof(id.internal));
  return HREC_OK;
}

extern "C" int hrec_comm_init(int rank, int world, const uint8_t* id, void** comm_out) {
  HREC_REQUIRE(id && comm_out, "comm_init: null pointer");
  HREC_REQUIRE(world >= 1 && rank >= 0 && rank < world, "comm_init: rank %d of world %d", rank, world);
  const Rccl* r = rccl();
  if (!r) {
    set_error("comm_init: librccl.so.1 could not be loaded");
    return HREC_E_UNSUPPORTED;
  }
  RcclId rid;
  memcpy(rid.internal, id, sizeof(rid.internal));
  void* nc = nullptr;
  const int rc = r->init(&nc, world, rid, rank);  // collective: every rank calls it
  if (rc) return rccl_fail(r, rc, "comm_init");
  *comm_out = new Comm{nc, rank, world};
  return HREC_OK;
}

extern "C" int hrec_comm_destroy(void* comm) {
  if (!comm) return HREC_OK;
  Comm* c = static_cast<Comm*>(comm);
  const Rccl* r = rccl();
  int rc = r ? r->destroy(c->nccl) : 0;
  delete c;
  if (rc) return rccl_fail(r, rc, "comm_destroy");
  return HREC_OK;
}

extern "C" int hrec_allgather(void* comm, const void* send, void* recv, size_t count, int dtype, void* stream) {
  HREC_REQUIRE(comm, "allgather: null communicator");
  HREC_REQUIRE(dtype >= 0 && dtype <= 4, "allgather: dtype must be 0 (f32), 1 (f64), 2 (i32), 3 (i64) or 4 (u8)");
  if (count == 0) return HREC_OK;
  HREC_REQUIRE(send && recv, "allgather: null buffer");
  static const int kRcclType[5] = {7 /* ncclFloat32 */, 8 /* ncclFloat64 */, 2 /* ncclInt32 */, 4 /* ncclInt64 */,
                                   1 /* ncclUint8 */};
  const Comm* c = static_cast<const Comm*>(comm);
  const Rccl* r = rccl();
  const int rc = r->allgather(send, recv, count, kRcclType[dtype], c->nccl, as_stream(stream));
  if (rc) return rccl_fail(r, rc, "allgather");
  return HREC_OK;
}

extern "C" int hrec_allreduce_minmax(void* comm, float* mm, int n_rows, int64_t n_users, void* stream) {
  HREC_REQUIRE(comm, "allreduce_minmax: null communicator");
  HREC_REQUIRE(n_rows >= 1 && n_users >= 0, "allreduce_minmax: bad shape");
  if (n_users == 0) return HREC_OK;
  HREC_REQUIRE(mm, "allreduce_minmax: null buffer");
  const Comm* c = static_cast<const Comm*>(comm);
  const Rccl* r = rccl();
  hipStream_t s = as_stream(stream);
  // rows 2m (minima) stay, rows 2m + 1 (maxima) are negated: one MIN over all
  const int64_t n = (int64_t)2 * n_rows * n_users;
  for (int m = 0; m < n_rows; ++m) {
    const int e = negate_rows(mm + ((int64_t)2 * m + 1) * n_users, n_users, s);
    if (e) return e;
  }
  const int rc = r->allreduce(mm, mm, (size_t)n, 7 /* ncclFloat32 */, 3 /* ncclMin */, c->nccl, s);
  if (rc) return rccl_fail(r, rc, "allreduce_minmax");
  for (int m = 0; m < n_rows; ++m) {
    const int e = negate_rows(mm + ((int64_t)2 * m + 1) * n_users, n_users, s);
    if (e) return e;
  }
  return HREC_OK;
}
