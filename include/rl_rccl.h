/*
 * rl_rccl.h — the RCCL transport for the multi-GPU router (include/rl_engine.h,
 * rl_router_*): one RCCL communicator over xGMI per router, all-to-all as grouped
 * ncclSend / ncclRecv of byte segments. Kept in its own library (librl_rccl.so) so the
 * engine's C-ABI does not depend on RCCL.
 *
 * Bootstrap: rank 0 calls rl_rccl_unique_id and hands the 128 bytes to every rank by the
 * caller's own channel (the JVM side, MPI, torch.distributed ...); every rank then calls
 * rl_transport_rccl_create with the same id (collective).
 */
#ifndef RL_RCCL_H
#define RL_RCCL_H

#include "rl_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RL_RCCL_ID_BYTES 128

int  rl_rccl_unique_id(void* id_out /* RL_RCCL_ID_BYTES */);
/* device: the HIP device of this rank (-1: current). */
int  rl_transport_rccl_create(const void* id, uint32_t world, uint32_t rank, int device,
                              rl_transport* out);
void rl_transport_rccl_destroy(rl_transport* t);

#ifdef __cplusplus
}
#endif
#endif /* RL_RCCL_H */
