// Multi-GPU exchange for the C ABI: an RCCL communicator per rank and the
// all-gather of emitted blocks.  RCCL is resolved with dlopen on
// first use, so loading libgraphwalk never requires librccl, and a process
// that already holds an RCCL (e.g. torch's) shares that copy by soname.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "graphwalk.h"

struct gw_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  std::string err;
};

namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*get_error_string)(ncclResult_t) = nullptr;
  std::string load_error;
};

const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      api.load_error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
      return;
    }
    api.get_unique_id = reinterpret_cast<decltype(api.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    api.comm_init_rank = reinterpret_cast<decltype(api.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    api.all_gather = reinterpret_cast<decltype(api.all_gather)>(dlsym(h, "ncclAllGather"));
    api.comm_destroy = reinterpret_cast<decltype(api.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    api.get_error_string = reinterpret_cast<decltype(api.get_error_string)>(dlsym(h, "ncclGetErrorString"));
    if (!api.get_unique_id || !api.comm_init_rank || !api.all_gather || !api.comm_destroy || !api.get_error_string)
      api.load_error = "librccl.so.1 lacks an ncclGetUniqueId/CommInitRank/AllGather/CommDestroy symbol";
  });
  return api;
}

thread_local std::string t_err;  // errors before a communicator exists

int fail_global(int code, const std::string& msg) {
  t_err = msg;
  return code;
}

std::string rccl_msg(const char* what, ncclResult_t r) {
  return std::string(what) + ": " + rccl().get_error_string(r);
}

}  // namespace

extern "C" {

int gw_comm_unique_id(uint8_t* id) {
  if (!id) return fail_global(GW_ERR_INVALID, "NULL id buffer");
  const RcclApi& a = rccl();
  if (!a.load_error.empty()) return fail_global(GW_ERR_DEVICE, a.load_error);
  ncclUniqueId u;
  const ncclResult_t r = a.get_unique_id(&u);
  if (r != ncclSuccess) return fail_global(GW_ERR_DEVICE, rccl_msg("ncclGetUniqueId", r));
  static_assert(sizeof(ncclUniqueId) == GW_COMM_ID_BYTES, "unique id size");
  std::memcpy(id, &u, GW_COMM_ID_BYTES);
  return GW_OK;
}

int gw_comm_init(const uint8_t* id, int nranks, int rank, int device, gw_comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks || device < 0)
    return fail_global(GW_ERR_INVALID, "bad arguments");
  *out = nullptr;
  const RcclApi& a = rccl();
  if (!a.load_error.empty()) return fail_global(GW_ERR_DEVICE, a.load_error);
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device >= count)
    return fail_global(GW_ERR_DEVICE, "device " + std::to_string(device) + " not visible");
  if (hipSetDevice(device) != hipSuccess) return fail_global(GW_ERR_DEVICE, "hipSetDevice failed");
  ncclUniqueId u;
  std::memcpy(&u, id, GW_COMM_ID_BYTES);
  gw_comm* c = new gw_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  const ncclResult_t r = a.comm_init_rank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail_global(GW_ERR_DEVICE, rccl_msg("ncclCommInitRank", r));
  }
  *out = c;
  return GW_OK;
}

int gw_comm_allgather(gw_comm* c, const void* send_dev, void* recv_dev, int64_t count, int dtype, void* stream) {
  if (!c) return fail_global(GW_ERR_INVALID, "NULL communicator");
  if (count < 0 || (count > 0 && (!send_dev || !recv_dev)) || (dtype != GW_DTYPE_I32 && dtype != GW_DTYPE_F64)) {
    c->err = "bad arguments";
    return GW_ERR_INVALID;
  }
  if (count == 0) return GW_OK;
  if (hipSetDevice(c->device) != hipSuccess) {
    c->err = "hipSetDevice failed";
    return GW_ERR_DEVICE;
  }
  const ncclDataType_t t = dtype == GW_DTYPE_I32 ? ncclInt32 : ncclFloat64;
  const ncclResult_t r = rccl().all_gather(send_dev, recv_dev, (size_t)count, t, c->comm, (hipStream_t)stream);
  if (r != ncclSuccess) {
    c->err = rccl_msg("ncclAllGather", r);
    return GW_ERR_DEVICE;
  }
  return GW_OK;
}

int gw_comm_free(gw_comm* c) {
  if (!c) return GW_OK;
  if (c->comm) (void)rccl().comm_destroy(c->comm);
  delete c;
  return GW_OK;
}

const char* gw_comm_last_error(const gw_comm* c) { return c ? c->err.c_str() : t_err.c_str(); }

}  // extern "C"
