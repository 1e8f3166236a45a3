// Monte-Carlo aggregation across GPUs: one RCCL communicator per process
// (one process per GPU) and a sum all-reduce of int64 error counters over
// xGMI.  The reference has no multi-process path (independent processes per
// sim_id, ldpc_jossy/py/ldpc_awgn.py:125-131); this is the single collective
// the decoding engine needs.  The unique id is produced by
// rank 0 and handed to the other ranks over the host rendezvous
// (ldpc_sparc_amd/rendezvous.py: standard-library TCP, no PyTorch).
#include <rccl/rccl.h>

#include <cstring>

#include "common.hpp"

struct sg_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1, device = 0;
};

#define SG_NCCL(call)                                                                              \
    do {                                                                                           \
        ncclResult_t r_ = (call);                                                                  \
        if (r_ != ncclSuccess)                                                                     \
            return ::sg::fail(SG_ERR_COMM, "%s failed: %s", #call, ncclGetErrorString(r_));        \
    } while (0)

extern "C" {

int sg_comm_unique_id(void *id_out) {
    SG_CHECK_ARG(id_out, "id_out is NULL");
    ncclUniqueId id;
    SG_NCCL(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof id);
    return SG_OK;
}

int sg_comm_init(int nranks, int rank, const void *id, sg_comm **out) {
    SG_CHECK_ARG(id && out, "null argument");
    SG_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank %d of %d", rank, nranks);
    SG_TRY(sg::ensure_device());
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    sg_comm *c = new sg_comm();
    hipGetDevice(&c->device);
    c->rank = rank;
    c->nranks = nranks;
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        return sg::fail(SG_ERR_COMM, "ncclCommInitRank failed: %s", ncclGetErrorString(r));
    }
    *out = c;
    return SG_OK;
}

int sg_comm_allreduce_sum_i64(sg_comm *c, int64_t *d_buf, size_t count, void *stream) {
    SG_CHECK_ARG(c && d_buf, "null argument");
    SG_NCCL(ncclAllReduce(d_buf, d_buf, count, ncclInt64, ncclSum, c->comm,
                          sg::pick_stream(stream)));
    return SG_OK;
}

// Number of ranks and this rank's device as RCCL sees them (ncclCommCount,
// ncclCommCuDevice): bench.py reports the rank count RCCL saw, not the one
// it asked for.
int sg_comm_info(sg_comm *c, int *nranks, int *device) {
    SG_CHECK_ARG(c && nranks && device, "null argument");
    SG_NCCL(ncclCommCount(c->comm, nranks));
    SG_NCCL(ncclCommCuDevice(c->comm, device));
    return SG_OK;
}

int sg_comm_destroy(sg_comm *c) {
    if (!c) return SG_OK;
    if (c->comm) ncclCommDestroy(c->comm);
    delete c;
    return SG_OK;
}

}  // extern "C"
