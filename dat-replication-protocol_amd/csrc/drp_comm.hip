// drp_comm.hip — the multi-GPU global frame index over RCCL.
//
// Independent replication streams are sharded across GPUs (contiguous blocks of stream ids,
// one process per GPU or one process driving several); each GPU decodes its block and turns
// the per-stream results into 32-byte drp_stream_stats records. The only collective of the
// whole codec is this one: an ncclAllGather (RCCL over xGMI) of those records, followed on
// every GPU by an exclusive scan of the frame counts (drp_index_scan), which gives every
// stream the global index of its first frame. A few KiB per GPU: latency-bound, no bulk data
// ever crosses GPUs.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <new>

#include "../../include/drp.h"

struct drp_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
};

static_assert(sizeof(ncclUniqueId) <= DRP_COMM_ID_BYTES, "unique id does not fit");

namespace {
int nccl_rc(ncclResult_t r) { return r == ncclSuccess ? DRP_OK : DRP_E_COMM; }
}  // namespace

extern "C" {

int drp_comm_id(uint8_t *id) {
  if (!id) return DRP_E_INVAL;
  ncclUniqueId u;
  const int rc = nccl_rc(ncclGetUniqueId(&u));
  if (rc != DRP_OK) return rc;
  memset(id, 0, DRP_COMM_ID_BYTES);
  memcpy(id, &u, sizeof u);
  return DRP_OK;
}

int drp_comm_init_rank(drp_ctx *ctx, const uint8_t *id, int nranks, int rank, drp_comm **out) {
  if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return DRP_E_INVAL;
  *out = nullptr;
  drp_comm *c = new (std::nothrow) drp_comm();
  if (!c) return DRP_E_NOMEM;
  c->device = drp_device(ctx);
  if (hipSetDevice(c->device) != hipSuccess) {
    delete c;
    return DRP_E_HIP;
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  const int rc = nccl_rc(ncclCommInitRank(&c->comm, nranks, u, rank));
  if (rc != DRP_OK) {
    delete c;
    return rc;
  }
  c->nranks = nranks;
  c->rank = rank;
  *out = c;
  return DRP_OK;
}

int drp_comm_init_all(drp_ctx **ctxs, int ngpu, drp_comm **comms) {
  if (!ctxs || !comms || ngpu < 1 || ngpu > 64) return DRP_E_INVAL;
  int devs[64];
  ncclComm_t raw[64];
  for (int g = 0; g < ngpu; g++) {
    if (!ctxs[g]) return DRP_E_INVAL;
    devs[g] = drp_device(ctxs[g]);
    comms[g] = nullptr;
  }
  const int rc = nccl_rc(ncclCommInitAll(raw, ngpu, devs));
  if (rc != DRP_OK) return rc;
  for (int g = 0; g < ngpu; g++) {
    comms[g] = new (std::nothrow) drp_comm();
    if (!comms[g]) {
      for (int k = 0; k < ngpu; k++) {
        if (k < g) delete comms[k];
        ncclCommDestroy(raw[k]);
        comms[k] = nullptr;
      }
      return DRP_E_NOMEM;
    }
    comms[g]->comm = raw[g];
    comms[g]->nranks = ngpu;
    comms[g]->rank = g;
    comms[g]->device = devs[g];
  }
  return DRP_OK;
}

void drp_comm_destroy(drp_comm *c) {
  if (!c) return;
  if (c->comm) {
    (void)hipSetDevice(c->device);
    ncclCommDestroy(c->comm);
  }
  delete c;
}

// One rank (process) of the all-gather: `local` holds this rank's per_rank records (pad a short
// block with zero records), `global` receives nranks * per_rank records in rank order and
// base[r * per_rank + i] the global index of rank r's i-th stream. Device pointers; returns
// after completion.
int drp_index_allgather(drp_ctx *ctx, drp_comm *comm, const drp_stream_stats *local, uint64_t per_rank,
                        drp_stream_stats *global, uint64_t *base) {
  if (!ctx || !comm || (per_rank && (!local || !global || !base))) return DRP_E_INVAL;
  if (drp_device(ctx) != comm->device) return DRP_E_INVAL;
  if (hipSetDevice(comm->device) != hipSuccess) return DRP_E_HIP;
  hipStream_t st = (hipStream_t)drp_stream(ctx);
  const size_t words = per_rank * (sizeof(drp_stream_stats) / sizeof(uint64_t));
  if (words) {
    int rc = nccl_rc(ncclAllGather(local, global, words, ncclUint64, comm->comm, st));
    if (rc != DRP_OK) return rc;
    rc = drp_index_scan(ctx, global, per_rank * (uint64_t)comm->nranks, base);
    if (rc != DRP_OK) return rc;
  }
  return drp_synchronize(ctx);
}

// The same for one process driving ngpu devices (a comm from drp_comm_init_all per device):
// one grouped all-gather, then the index scan on every device.
int drp_index_allgather_multi(drp_ctx **ctxs, drp_comm **comms, int ngpu, const drp_stream_stats *const *local,
                              uint64_t per_gpu, drp_stream_stats *const *global, uint64_t *const *base) {
  if (!ctxs || !comms || ngpu < 1 || (per_gpu && (!local || !global || !base))) return DRP_E_INVAL;
  const size_t words = per_gpu * (sizeof(drp_stream_stats) / sizeof(uint64_t));
  if (!words) return DRP_OK;
  for (int g = 0; g < ngpu; g++)
    if (!ctxs[g] || !comms[g] || drp_device(ctxs[g]) != comms[g]->device) return DRP_E_INVAL;
  int rc = nccl_rc(ncclGroupStart());
  if (rc != DRP_OK) return rc;
  for (int g = 0; g < ngpu; g++) {
    if (hipSetDevice(comms[g]->device) != hipSuccess) {
      ncclGroupEnd();
      return DRP_E_HIP;
    }
    rc = nccl_rc(ncclAllGather(local[g], global[g], words, ncclUint64, comms[g]->comm,
                               (hipStream_t)drp_stream(ctxs[g])));
    if (rc != DRP_OK) {
      ncclGroupEnd();
      return rc;
    }
  }
  rc = nccl_rc(ncclGroupEnd());
  if (rc != DRP_OK) return rc;
  for (int g = 0; g < ngpu; g++) {
    rc = drp_index_scan(ctxs[g], global[g], per_gpu * (uint64_t)ngpu, base[g]);
    if (rc != DRP_OK) return rc;
  }
  for (int g = 0; g < ngpu; g++) {
    rc = drp_synchronize(ctxs[g]);
    if (rc != DRP_OK) return rc;
  }
  return DRP_OK;
}

int drp_index_allgather_host(drp_ctx **ctxs, drp_comm **comms, int ngpu, const drp_stream_stats *const *local,
                             uint64_t per_gpu, drp_stream_stats *global, uint64_t *base) {
  if (!ctxs || !comms || ngpu < 1 || ngpu > 64 || (per_gpu && (!local || !global || !base))) return DRP_E_INVAL;
  if (!per_gpu) return DRP_OK;
  const size_t lb = per_gpu * sizeof(drp_stream_stats), gb = lb * (size_t)ngpu, bb = per_gpu * (size_t)ngpu * 8;
  void *dl[64] = {}, *dg[64] = {}, *db[64] = {};
  int rc = DRP_OK;
  for (int g = 0; g < ngpu && rc == DRP_OK; g++) {
    if (!ctxs[g] || !local[g] || hipSetDevice(drp_device(ctxs[g])) != hipSuccess) {
      rc = !ctxs[g] || !local[g] ? DRP_E_INVAL : DRP_E_HIP;
      break;
    }
    if (hipMalloc(&dl[g], lb) != hipSuccess || hipMalloc(&dg[g], gb) != hipSuccess || hipMalloc(&db[g], bb) != hipSuccess)
      rc = DRP_E_NOMEM;
    else if (hipMemcpyAsync(dl[g], local[g], lb, hipMemcpyHostToDevice, (hipStream_t)drp_stream(ctxs[g])) != hipSuccess)
      rc = DRP_E_HIP;
  }
  if (rc == DRP_OK)
    rc = drp_index_allgather_multi(ctxs, comms, ngpu, (const drp_stream_stats *const *)dl, per_gpu,
                                   (drp_stream_stats *const *)dg, (uint64_t *const *)db);
  if (rc == DRP_OK && hipSetDevice(drp_device(ctxs[0])) == hipSuccess) {
    if (hipMemcpy(global, dg[0], gb, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(base, db[0], bb, hipMemcpyDeviceToHost) != hipSuccess)
      rc = DRP_E_HIP;
  }
  for (int g = 0; g < ngpu; g++) {
    if (!ctxs[g]) continue;
    (void)hipSetDevice(drp_device(ctxs[g]));
    if (dl[g]) (void)hipFree(dl[g]);
    if (dg[g]) (void)hipFree(dg[g]);
    if (db[g]) (void)hipFree(db[g]);
  }
  return rc;
}

}  // extern "C"
