// rl_rccl.cpp — RCCL transport of the multi-GPU router (include/rl_rccl.h).
// One communicator per router; an all-to-all of byte segments is one group of
// ncclSend / ncclRecv (RCCL 2.27, /opt/rocm/include/rccl/rccl.h), peer segments of any
// size including zero and the rank itself.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>

#include "../../include/rl_rccl.h"

namespace {
struct Rccl {
    ncclComm_t comm = nullptr;
    int world = 0;
};

int a2av(void* ctx, const void* send, const uint64_t* so, const uint64_t* sb, void* recv,
         const uint64_t* ro, const uint64_t* rb, void* stream) {
    Rccl* c = (Rccl*)ctx;
    hipStream_t s = (hipStream_t)stream;
    if (ncclGroupStart() != ncclSuccess) return -1;
    for (int p = 0; p < c->world; ++p) {
        if (sb[p] && ncclSend((const char*)send + so[p], sb[p], ncclUint8, p, c->comm, s) != ncclSuccess) {
            (void)ncclGroupEnd();
            return -1;
        }
        if (rb[p] && ncclRecv((char*)recv + ro[p], rb[p], ncclUint8, p, c->comm, s) != ncclSuccess) {
            (void)ncclGroupEnd();
            return -1;
        }
    }
    return ncclGroupEnd() == ncclSuccess ? 0 : -1;
}
}  // namespace

static_assert(sizeof(ncclUniqueId) == RL_RCCL_ID_BYTES, "ncclUniqueId size");

extern "C" int rl_rccl_unique_id(void* id_out) {
    if (!id_out) return RL_E_INVALID_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return RL_E_DEVICE;
    std::memcpy(id_out, &id, sizeof(id));
    return RL_OK;
}

extern "C" int rl_transport_rccl_create(const void* id, uint32_t world, uint32_t rank, int device,
                                        rl_transport* out) {
    if (!id || !out || world == 0 || rank >= world) return RL_E_INVALID_ARG;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) return RL_E_DEVICE;
    Rccl* c = new (std::nothrow) Rccl();
    if (!c) return RL_E_NOMEM;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&c->comm, (int)world, u, (int)rank) != ncclSuccess) {
        delete c;
        return RL_E_DEVICE;
    }
    c->world = (int)world;
    out->ctx = c;
    out->all_to_all_v = a2av;
    return RL_OK;
}

extern "C" void rl_transport_rccl_destroy(rl_transport* t) {
    if (!t || !t->ctx) return;
    Rccl* c = (Rccl*)t->ctx;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
    t->ctx = nullptr;
    t->all_to_all_v = nullptr;
}
