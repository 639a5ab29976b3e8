// comm.hip — the multi-GPU exchange of the eval path as a C ABI over RCCL
// (the NCCL API on ROCm; xGMI between the GPUs of one node), for callers that are not Python.
// The Python drop-in does the same exchange through torch.distributed's "nccl" process group
// (multimodal_reid_amd/distributed.py); both move the same bytes in the same layout:
//   * gallery (and, for the re-rank, query) feature rows sharded contiguously over ranks,
//     rank r owning rows [n r / W, n (r+1) / W) (distributed.shard) -> one padded all-gather
//     + an in-order compaction (reidmi_comm_allgather_rows);
//   * per-query results, also by reidmi_comm_allgather_rows (so the host reduction runs in
//     global query order and CMC/mAP are bit-identical for every world size);
//   * reidmi_comm_allreduce for sums a caller wants reduced on the device.
// librccl.so.1 is opened at first use (dlopen): inside a process that already loaded torch it
// resolves to torch's copy (same soname), so there is one RCCL in the process; a C caller
// without RCCL installed still loads libreidmi.so (these calls then fail with a message).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "common.h"

struct reidmi_comm {
    ncclComm_t nc;
    int nranks, rank;
};

namespace reidmi {
namespace {
struct Rccl {
    bool tried = false, ok = false;
    std::string why;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) err_str = nullptr;
};
Rccl g_rccl;
std::mutex g_rccl_mu;

template <typename F>
bool sym(void* h, const char* name, F& f) {
    f = (F)dlsym(h, name);
    return f != nullptr;
}

const Rccl* rccl() {
    std::lock_guard<std::mutex> g(g_rccl_mu);
    if (!g_rccl.tried) {
        g_rccl.tried = true;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            g_rccl.why = std::string("librccl.so.1 not loadable: ") + (e ? e : "?");
        } else if (!(sym(h, "ncclGetUniqueId", g_rccl.get_unique_id) && sym(h, "ncclCommInitRank", g_rccl.init_rank) &&
                     sym(h, "ncclCommDestroy", g_rccl.destroy) && sym(h, "ncclAllGather", g_rccl.all_gather) &&
                     sym(h, "ncclAllReduce", g_rccl.all_reduce) && sym(h, "ncclGetErrorString", g_rccl.err_str))) {
            g_rccl.why = "librccl.so.1 lacks an NCCL entry point";
        } else {
            g_rccl.ok = true;
        }
    }
    return g_rccl.ok ? &g_rccl : nullptr;
}

int nccl_fail(const Rccl* r, ncclResult_t e, const char* what) {
    return fail(EHIP, std::string(what) + ": " + (r && r->err_str ? r->err_str(e) : "rccl error"));
}

#define RM_RCCL()                                                                 \
    const Rccl* R = rccl();                                                       \
    if (!R) return fail(EHIP, "RCCL unavailable (" + g_rccl.why + ")");

// rows of rank r under the contiguous shard (distributed.shard)
inline int64_t shard_lo(int64_t n, int r, int w) { return n * r / w; }
}  // namespace
}  // namespace reidmi

using namespace reidmi;

REIDMI_API int reidmi_comm_unique_id(void* id) {
    RM_REQUIRE(id, "comm_unique_id: null id");
    RM_RCCL();
    ncclUniqueId u;
    const ncclResult_t e = R->get_unique_id(&u);
    if (e != ncclSuccess) return nccl_fail(R, e, "ncclGetUniqueId");
    static_assert(sizeof(ncclUniqueId) == REIDMI_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, sizeof(u));
    return OK;
}

REIDMI_API int reidmi_comm_init(reidmi_comm_t* comm, int nranks, int rank, const void* id, int device) {
    RM_REQUIRE(comm && id && nranks >= 1 && rank >= 0 && rank < nranks && device >= 0, "comm_init: bad arguments");
    RM_RCCL();
    RM_CHECK_HIP(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t nc = nullptr;
    const ncclResult_t e = R->init_rank(&nc, nranks, u, rank);
    if (e != ncclSuccess) return nccl_fail(R, e, "ncclCommInitRank");
    *comm = new reidmi_comm{nc, nranks, rank};
    return OK;
}

REIDMI_API int reidmi_comm_destroy(reidmi_comm_t comm) {
    if (!comm) return OK;
    RM_RCCL();
    const ncclResult_t e = R->destroy(comm->nc);
    delete comm;
    if (e != ncclSuccess) return nccl_fail(R, e, "ncclCommDestroy");
    return OK;
}

REIDMI_API int reidmi_comm_rank(reidmi_comm_t comm, int* rank, int* nranks) {
    RM_REQUIRE(comm && rank && nranks, "comm_rank: bad arguments");
    *rank = comm->rank;
    *nranks = comm->nranks;
    return OK;
}

REIDMI_API int64_t reidmi_comm_allgather_rows_scratch_bytes(int nranks, int64_t n_total, int64_t row_bytes) {
    if (nranks < 1 || n_total < 0 || row_bytes <= 0) return -1;
    return (int64_t)nranks * ((n_total + nranks - 1) / nranks) * row_bytes;
}

REIDMI_API int reidmi_comm_allgather_rows(reidmi_comm_t comm, const void* send, int64_t n_total, int64_t row_bytes,
                                          void* recv, void* scratch, int64_t scratch_bytes, void* stream) {
    RM_REQUIRE(comm && recv && n_total >= 0 && row_bytes > 0, "comm_allgather_rows: bad arguments");
    const int W = comm->nranks, r = comm->rank;
    const int64_t mx = (n_total + W - 1) / W;
    RM_REQUIRE(scratch && scratch_bytes >= (int64_t)W * mx * row_bytes,
               "comm_allgather_rows: scratch of reidmi_comm_allgather_rows_scratch_bytes required");
    RM_RCCL();
    if (n_total == 0) return OK;
    hipStream_t s = (hipStream_t)stream;
    char* sc = (char*)scratch;
    const int64_t slot = mx * row_bytes;
    const int64_t mine = shard_lo(n_total, r + 1, W) - shard_lo(n_total, r, W);
    RM_REQUIRE(mine == 0 || send, "comm_allgather_rows: null send");
    // own rows into the rank's slot (in-place all-gather), the slot's tail is padding
    if (mine) RM_CHECK_HIP(hipMemcpyAsync(sc + r * slot, send, mine * row_bytes, hipMemcpyDeviceToDevice, s));
    const ncclResult_t e = R->all_gather(sc + r * slot, sc, (size_t)slot, ncclUint8, comm->nc, s);
    if (e != ncclSuccess) return nccl_fail(R, e, "ncclAllGather");
    // compaction in rank order: rows [lo_q, hi_q) of rank q
    for (int q = 0; q < W; q++) {
        const int64_t lo = shard_lo(n_total, q, W), n = shard_lo(n_total, q + 1, W) - lo;
        if (n) RM_CHECK_HIP(hipMemcpyAsync((char*)recv + lo * row_bytes, sc + q * slot, n * row_bytes,
                                           hipMemcpyDeviceToDevice, s));
    }
    return OK;
}

REIDMI_API int reidmi_comm_allreduce(reidmi_comm_t comm, const void* send, void* recv, int64_t count, int dtype,
                                     void* stream) {
    RM_REQUIRE(comm && send && recv && count >= 0 && dtype >= 0 && dtype <= 3, "comm_allreduce: bad arguments");
    RM_RCCL();
    if (count == 0) return OK;
    static const ncclDataType_t types[4] = {ncclFloat32, ncclFloat64, ncclInt32, ncclInt64};
    const ncclResult_t e = R->all_reduce(send, recv, (size_t)count, types[dtype], ncclSum, comm->nc, (hipStream_t)stream);
    if (e != ncclSuccess) return nccl_fail(R, e, "ncclAllReduce");
    return OK;
}
