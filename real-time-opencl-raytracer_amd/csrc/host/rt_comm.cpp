// rt_comm.cpp -- native band exchange for multi-GPU frames over RCCL (xGMI).
//
// The frame's one real exchange (the reference reads the frame back to the
// host, RayTracer.cpp:343) issued from C++ on the frame's own stream: ncclGather of every
// rank's band buffer into rank 0's slots, then (rank 0) rt_assemble_bands into the frame.
// Render, gather and assembly of one frame are then ordered by one stream with no
// cross-stream waits, and a frame costs the host three C calls.  A communicator serves one
// stream at a time (RCCL serialises a communicator's operations), so a caller with frames
// in flight creates one rt_comm per in-flight stream.  torch.distributed (or any other
// channel) only carries the 128-byte id from rank 0 to the others.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "rt_abi.h"

struct rt_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
};

static std::string g_comm_err;

static int comm_err(const std::string& m, int code) {
    g_comm_err = m;
    return code;
}

extern "C" {

const char* rt_comm_last_error(void) { return g_comm_err.c_str(); }

int rt_comm_unique_id(uint8_t* id, int32_t id_bytes) {
    if (!id || id_bytes < (int32_t)sizeof(ncclUniqueId)) return comm_err("rt_comm_unique_id: buffer", RT_ERR_INVALID_ARG);
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return comm_err(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r), RT_ERR_DEVICE);
    std::memcpy(id, &u, sizeof u);
    return RT_OK;
}

int rt_comm_create(int32_t device, int32_t nranks, int32_t rank, const uint8_t* id, int32_t id_bytes, rt_comm** out) {
    if (!out || !id || id_bytes < (int32_t)sizeof(ncclUniqueId) || nranks < 1 || rank < 0 || rank >= nranks)
        return comm_err("rt_comm_create: invalid argument", RT_ERR_INVALID_ARG);
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return comm_err("rt_comm_create: hipSetDevice", RT_ERR_DEVICE);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    rt_comm* c = new rt_comm();
    const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return comm_err(std::string("ncclCommInitRank: ") + ncclGetErrorString(r), RT_ERR_DEVICE);
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *out = c;
    return RT_OK;
}

int rt_comm_destroy(rt_comm* c) {
    if (!c) return RT_ERR_INVALID_ARG;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
    return RT_OK;
}

int rt_frame_gather(rt_comm* c, const uint32_t* d_bands, uint64_t slot_pixels, uint32_t* d_slots, uint32_t* d_frame,
                    uint32_t w, uint32_t h, int32_t band_rows, void* stream) {
    if (!c || !d_bands || slot_pixels == 0 || w == 0 || h == 0 || band_rows < 1)
        return comm_err("rt_frame_gather: invalid argument", RT_ERR_INVALID_ARG);
    if (c->rank == 0 && (!d_slots || !d_frame)) return comm_err("rt_frame_gather: rank 0 needs slots and frame", RT_ERR_INVALID_ARG);
    const ncclResult_t r = ncclGather(d_bands, c->rank == 0 ? d_slots : nullptr, slot_pixels, ncclUint32, 0, c->comm,
                                      (hipStream_t)stream);
    if (r != ncclSuccess) return comm_err(std::string("ncclGather: ") + ncclGetErrorString(r), RT_ERR_DEVICE);
    if (c->rank == 0) {
        const int rc = rt_assemble_bands(d_frame, d_slots, slot_pixels, w, h, c->nranks, band_rows, stream);
        if (rc) return comm_err(std::string("rt_assemble_bands: ") + rt_last_error(nullptr), rc);
    }
    return RT_OK;
}

}  // extern "C"
