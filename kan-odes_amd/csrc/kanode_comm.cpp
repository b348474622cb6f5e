// kanode_comm.cpp — the data-parallel gradient all-reduce for hosts without a collective of their own.
//
// The reference trains one model per process (Lotka-Volterra/LV_driver_KANODE.jl:219-291,
// PDE examples/Fisher-KPP_Source.jl:163-213: Flux `update!` after Zygote's gradient); the MI355X
// layout is one process per GPU, each with a trajectory shard, and ONE all-reduce of the flat
// [dp; L] vector per optimiser step.  Python drivers do that all-reduce with
// torch.distributed (backend "nccl" = RCCL).  A Julia or C driver links only libkanode.so, so the
// library carries the same step as a C-ABI over RCCL: a communicator per process (its unique id made
// by rank 0 and handed to the others by the host: a file, MPI.jl, an environment variable) and an
// in-place SUM all-reduce on the handle's stream, followed by kanode_adam_step with scale =
// 1/nranks (the mean gradient, kanode/train.py).  RCCL picks the xGMI ring/tree itself.
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include <hip/hip_runtime.h>

#include "kanode.h"

struct kanode_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    std::string err;
};

namespace {

thread_local std::string g_comm_err;   // failures with no communicator to hold the message

kanode_status comm_fail(kanode_comm* c, kanode_status s, const std::string& msg) {
    (c ? c->err : g_comm_err) = msg;
    return s;
}

}  // namespace

extern "C" {

kanode_status kanode_comm_unique_id(uint8_t* id) {
    if (!id) return comm_fail(nullptr, KANODE_ERR_INVALID_ARG, "kanode_comm_unique_id: id is NULL");
    static_assert(sizeof(ncclUniqueId) == KANODE_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return comm_fail(nullptr, KANODE_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(id, &u, sizeof(u));
    return KANODE_OK;
}

kanode_status kanode_comm_create(int32_t nranks, int32_t rank, const uint8_t* id, int32_t device, kanode_comm** out) {
    if (!out) return comm_fail(nullptr, KANODE_ERR_INVALID_ARG, "kanode_comm_create: out is NULL");
    *out = nullptr;
    if (!id) return comm_fail(nullptr, KANODE_ERR_INVALID_ARG, "kanode_comm_create: id is NULL");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return comm_fail(nullptr, KANODE_ERR_INVALID_ARG,
                         "kanode_comm_create: need 0 <= rank < nranks, got rank " + std::to_string(rank) +
                             " of " + std::to_string(nranks));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        (void)hipGetLastError();
        return comm_fail(nullptr, KANODE_ERR_INVALID_ARG,
                         "kanode_comm_create: device " + std::to_string(device) + " not present (" +
                             std::to_string(ndev) + " visible)");
    }
    // RCCL binds the communicator to the calling thread's current device; the caller's (Julia's, torch's)
    // current device is put back afterwards.  One rank per GPU: RCCL refuses two on one device.
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return comm_fail(nullptr, KANODE_ERR_HIP, "kanode_comm_create: hipGetDevice / hipSetDevice failed");
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    auto* c = new kanode_comm();
    const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
    (void)hipSetDevice(prev);
    if (r != ncclSuccess) {
        delete c;
        return comm_fail(nullptr, KANODE_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *out = c;
    return KANODE_OK;
}

kanode_status kanode_comm_allreduce_sum(kanode_comm* c, void* buf, int64_t count, int32_t dtype, void* stream) {
    if (!c) return comm_fail(nullptr, KANODE_ERR_INVALID_ARG, "kanode_comm_allreduce_sum: null communicator");
    if (count < 0 || (count > 0 && !buf)) return comm_fail(c, KANODE_ERR_INVALID_ARG, "kanode_comm_allreduce_sum: bad buffer");
    if (dtype != KANODE_F32 && dtype != KANODE_F64)
        return comm_fail(c, KANODE_ERR_INVALID_ARG, "kanode_comm_allreduce_sum: dtype must be KANODE_F32 or KANODE_F64");
    if (count == 0) return KANODE_OK;
    const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, dtype == KANODE_F64 ? ncclFloat64 : ncclFloat32, ncclSum,
                                         c->comm, (hipStream_t)stream);
    if (r != ncclSuccess) return comm_fail(c, KANODE_ERR_HIP, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    return KANODE_OK;
}

int32_t kanode_comm_size(const kanode_comm* c) { return c ? c->nranks : -1; }
int32_t kanode_comm_rank(const kanode_comm* c) { return c ? c->rank : -1; }

const char* kanode_comm_last_error(const kanode_comm* c) { return c ? c->err.c_str() : g_comm_err.c_str(); }

void kanode_comm_destroy(kanode_comm* c) {
    if (!c) return;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
}

}  // extern "C"
