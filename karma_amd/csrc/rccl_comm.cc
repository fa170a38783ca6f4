// karma_amd/csrc/rccl_comm.cc -- the engine's RCCL communicator (one process
// per GPU, xGMI) for the multi-GPU path: unique id, init/destroy, and the
// gather of per-record CRCs to the root.
//
// RCCL is bound at run time through ONE library handle.  A process may already
// hold an RCCL (PyTorch ships its own librccl); linking ours as well would
// let the dynamic linker resolve each nccl* symbol from whichever copy comes
// first in scope, mixing two RCCLs on one communicator.  So: reuse an RCCL that
// is already loaded (RTLD_NOLOAD), else load ROCm's, and take every entry
// point from that handle.  The gather uses ncclGather when the library has it
// and a grouped ncclSend/ncclRecv otherwise.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "gather_p2p.h"
#include "karma_crc32c.h"

namespace karma::engine {
int set_last_error(int code, const std::string& what);  // capi.cc
}

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*commCount)(const ncclComm_t, int*) = nullptr;
    const char* (*getErrorString)(ncclResult_t) = nullptr;
    ncclResult_t (*gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)() = nullptr;
    ncclResult_t (*groupEnd)() = nullptr;
    std::string error;
};

template <typename F>
void bind(void* h, F& f, const char* name) {
    f = reinterpret_cast<F>(dlsym(h, name));
}

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {"librccl.so.1", "librccl.so"};
        for (const char* n : names)
            if ((r.h = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;  // an RCCL already in the process
        if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!r.h) r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!r.h) {
            const char* e = dlerror();
            r.error = std::string("cannot load librccl: ") + (e ? e : "?");
            return;
        }
        bind(r.h, r.getUniqueId, "ncclGetUniqueId");
        bind(r.h, r.commInitRank, "ncclCommInitRank");
        bind(r.h, r.commDestroy, "ncclCommDestroy");
        bind(r.h, r.commCount, "ncclCommCount");
        bind(r.h, r.getErrorString, "ncclGetErrorString");
        bind(r.h, r.gather, "ncclGather");
        bind(r.h, r.send, "ncclSend");
        bind(r.h, r.recv, "ncclRecv");
        bind(r.h, r.groupStart, "ncclGroupStart");
        bind(r.h, r.groupEnd, "ncclGroupEnd");
        if (!r.getUniqueId || !r.commInitRank || !r.commDestroy || !r.getErrorString ||
            (!r.gather && !(r.send && r.recv && r.groupStart && r.groupEnd))) {
            r.error = "librccl lacks a required entry point";
            r.h = nullptr;
        }
    });
    return r;
}

int rfail(const std::string& what) { return karma::engine::set_last_error(KARMA_E_RCCL, what); }

}  // namespace

struct karma_comm {
    ncclComm_t nc = nullptr;
    int rank = 0, nranks = 1;
};

extern "C" {

int karma_crc32c_get_unique_id(void* uid, size_t uid_bytes) {
    if (!uid || uid_bytes < sizeof(ncclUniqueId)) return KARMA_E_INVALID;
    Rccl& r = rccl();
    if (!r.h) return rfail(r.error);
    ncclUniqueId id;
    const ncclResult_t e = r.getUniqueId(&id);
    if (e != ncclSuccess) return rfail(std::string("ncclGetUniqueId: ") + r.getErrorString(e));
    std::memcpy(uid, &id, sizeof(id));
    return 0;
}

int karma_crc32c_comm_init(karma_comm_t* comm, int nranks, const void* uid, int rank) {
    if (!comm || !uid || nranks < 1 || rank < 0 || rank >= nranks) return KARMA_E_INVALID;
    Rccl& r = rccl();
    if (!r.h) return rfail(r.error);
    karma_comm* c = new (std::nothrow) karma_comm;
    if (!c) return KARMA_E_NOMEM;
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    const ncclResult_t e = r.commInitRank(&c->nc, nranks, id, rank);
    if (e != ncclSuccess) {
        delete c;
        return rfail(std::string("ncclCommInitRank: ") + r.getErrorString(e));
    }
    c->rank = rank;
    c->nranks = nranks;
    *comm = c;
    return 0;
}

int karma_crc32c_comm_destroy(karma_comm_t comm) {
    if (!comm) return 0;
    Rccl& r = rccl();
    const ncclResult_t e = r.h ? r.commDestroy(comm->nc) : ncclSuccess;
    delete comm;
    if (e != ncclSuccess) return rfail(std::string("ncclCommDestroy: ") + r.getErrorString(e));
    return 0;
}

int karma_crc32c_comm_count(karma_comm_t comm, int* nranks) {
    if (!comm || !nranks) return KARMA_E_INVALID;
    Rccl& r = rccl();
    if (!r.h) return rfail(r.error);
    if (!r.commCount) {  // an RCCL without ncclCommCount: the size the communicator was built with
        *nranks = comm->nranks;
        return 0;
    }
    const ncclResult_t e = r.commCount(comm->nc, nranks);
    if (e != ncclSuccess) return rfail(std::string("ncclCommCount: ") + r.getErrorString(e));
    return 0;
}

int karma_crc32c_gather_u32(karma_comm_t comm, const uint32_t* d_send, size_t count, uint32_t* d_recv, int root,
                            karma_stream_t stream) {
    if (!comm || (!d_send && count) || root < 0 || root >= comm->nranks) return KARMA_E_INVALID;
    if (comm->rank == root && !d_recv && count) return KARMA_E_INVALID;
    Rccl& r = rccl();
    if (!r.h) return rfail(r.error);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (r.gather) {
        const ncclResult_t e = r.gather(d_send, d_recv, count, ncclUint32, root, comm->nc, s);
        if (e != ncclSuccess) return rfail(std::string("ncclGather: ") + r.getErrorString(e));
        return 0;
    }
    // grouped point-to-point form (gather_p2p.h): every rank sends, the root receives each
    // shard in rank order and copies its own
    struct Ops {
        Rccl& r;
        karma_comm* c;
        hipStream_t s;
        ncclResult_t last = ncclSuccess;
        int nc(ncclResult_t e) {
            if (e != ncclSuccess) last = e;
            return e != ncclSuccess ? KARMA_E_RCCL : 0;
        }
        int group_start() { return nc(r.groupStart()); }
        int group_end() { return nc(r.groupEnd()); }
        int send(const uint32_t* b, size_t n, int peer) { return nc(r.send(b, n, ncclUint32, peer, c->nc, s)); }
        int recv(uint32_t* b, size_t n, int peer) { return nc(r.recv(b, n, ncclUint32, peer, c->nc, s)); }
        int copy(uint32_t* d, const uint32_t* src, size_t n) {
            return hipMemcpyAsync(d, src, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s) == hipSuccess ? 0
                                                                                                 : KARMA_E_HIP;
        }
    } ops{r, comm, s};
    const int rc = karma::engine::gather_p2p(ops, comm->rank, comm->nranks, root, d_send, count, d_recv);
    if (rc == KARMA_E_RCCL) return rfail(std::string("ncclSend/ncclRecv: ") + r.getErrorString(ops.last));
    if (rc) return karma::engine::set_last_error(rc, "gather_u32: root's own copy");
    return 0;
}

}  // extern "C"
