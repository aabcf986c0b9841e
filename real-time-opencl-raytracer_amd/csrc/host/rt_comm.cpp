// rt_comm.cpp -- native band exchange for multi-GPU frames over RCCL (xGMI).
//
// The frame's one real exchange (the reference reads the frame back to the
// host, RayTracer.cpp:343), issued from C++: ncclGather of every rank's band buffer into
// rank 0's slots, then (rank 0) rt_assemble_bands into the frame.
//
// rt_frame_exchange (the bench path): ONE communicator per rank, its gathers in issue order
// on the communicator's own stream, rank 0's assemblies on a second stream; the frame's
// render stream is joined to them by events only.  The caller cycles buffer sets ("slots"):
// a frame's render into slot j waits (rt_frame_slot_wait) only for the gather that last read
// slot j, issued several frames earlier, so render streams never wait on the latest gather.
// A frame costs the host three C calls (render, slot wait, exchange).
//
// rt_frame_gather: the same exchange on the caller's stream (one stream per communicator).
// torch.distributed (or any other channel) only carries the 128-byte id from rank 0.
//
// rt_bands_put (bench.py --gather ipc): no collective at all.  Rank 0's framebuffers are
// exported once as a HIP IPC handle (rt_ipc_alloc / rt_ipc_open); every rank then copies its
// bands straight to their rows of rank 0's frame with one small copy kernel per frame on its
// own stream (rt_bands_put, rt_render.hip).  Over xGMI the copy runs on the sending GPU; rank
// 0 runs no receive kernel and no re-interleave, and no kernel anywhere spins waiting for a
// peer.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "rt_abi.h"

struct rt_comm {
    static constexpr int kSlots = 64;
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    hipStream_t xs = nullptr;   // gathers, in issue order
    hipStream_t xa = nullptr;   // rank 0: assemblies
    hipEvent_t ready[kSlots] = {}, gathered[kSlots] = {}, assembled[kSlots] = {};
    bool sent[kSlots] = {}, built[kSlots] = {};
};

static void comm_release(rt_comm* c) {
    for (int i = 0; i < rt_comm::kSlots; ++i) {
        if (c->ready[i]) (void)hipEventDestroy(c->ready[i]);
        if (c->gathered[i]) (void)hipEventDestroy(c->gathered[i]);
        if (c->assembled[i]) (void)hipEventDestroy(c->assembled[i]);
    }
    if (c->xs) (void)hipStreamDestroy(c->xs);
    if (c->xa) (void)hipStreamDestroy(c->xa);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
}

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
    // the exchange streams at the device's highest priority: a gather or assembly is a few
    // workgroups that should not queue behind the next frame's render waves
    int lo = 0, hi = 0;
    bool ok = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
              hipStreamCreateWithPriority(&c->xs, hipStreamNonBlocking, hi) == hipSuccess &&
              hipStreamCreateWithPriority(&c->xa, hipStreamNonBlocking, hi) == hipSuccess;
    for (int i = 0; ok && i < rt_comm::kSlots; ++i)
        ok = hipEventCreateWithFlags(&c->ready[i], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&c->gathered[i], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&c->assembled[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        comm_release(c);
        return comm_err("rt_comm_create: exchange streams / events", RT_ERR_DEVICE);
    }
    *out = c;
    return RT_OK;
}

int rt_comm_destroy(rt_comm* c) {
    if (!c) return RT_ERR_INVALID_ARG;
    (void)hipSetDevice(c->device);
    if (c->xs) (void)hipStreamSynchronize(c->xs);
    if (c->xa) (void)hipStreamSynchronize(c->xa);
    comm_release(c);
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

int rt_frame_exchange(rt_comm* c, int32_t slot, int32_t nframes, const uint32_t* d_bands, uint64_t frame_pixels,
                      uint32_t* d_slots, uint32_t* d_frames, uint32_t w, uint32_t h, int32_t band_rows, void* stream) {
    if (!c || slot < 0 || slot >= rt_comm::kSlots || nframes < 1 || !d_bands || frame_pixels == 0 || w == 0 || h == 0 ||
        band_rows < 1)
        return comm_err("rt_frame_exchange: invalid argument", RT_ERR_INVALID_ARG);
    const bool root = c->rank == 0;
    if (root && (!d_slots || !d_frames)) return comm_err("rt_frame_exchange: rank 0 needs slots and frames", RT_ERR_INVALID_ARG);
    const uint64_t slot_pixels = (uint64_t)nframes * frame_pixels;   // one rank's share of the gather
    // the gather after the frames' renders; on rank 0 also after the slot's previous assembly
    // (it read d_slots)
    if (hipEventRecord(c->ready[slot], (hipStream_t)stream) != hipSuccess ||
        hipStreamWaitEvent(c->xs, c->ready[slot], 0) != hipSuccess ||
        (root && c->built[slot] && hipStreamWaitEvent(c->xs, c->assembled[slot], 0) != hipSuccess))
        return comm_err("rt_frame_exchange: stream ordering", RT_ERR_DEVICE);
    const ncclResult_t r = ncclGather(d_bands, root ? d_slots : nullptr, slot_pixels, ncclUint32, 0, c->comm, c->xs);
    if (r != ncclSuccess) return comm_err(std::string("ncclGather: ") + ncclGetErrorString(r), RT_ERR_DEVICE);
    if (hipEventRecord(c->gathered[slot], c->xs) != hipSuccess)
        return comm_err("rt_frame_exchange: event record", RT_ERR_DEVICE);
    c->sent[slot] = true;
    if (root) {
        if (hipStreamWaitEvent(c->xa, c->gathered[slot], 0) != hipSuccess)
            return comm_err("rt_frame_exchange: stream ordering", RT_ERR_DEVICE);
        const int rc = rt_assemble_bands_batch(d_frames, d_slots, slot_pixels, frame_pixels, nframes, w, h, c->nranks,
                                               band_rows, c->xa);
        if (rc) return comm_err(std::string("rt_assemble_bands: ") + rt_last_error(nullptr), rc);
        if (hipEventRecord(c->assembled[slot], c->xa) != hipSuccess)
            return comm_err("rt_frame_exchange: event record", RT_ERR_DEVICE);
        c->built[slot] = true;
    }
    return RT_OK;
}

int rt_frame_slot_wait(rt_comm* c, int32_t slot, void* stream) {
    if (!c || slot < 0 || slot >= rt_comm::kSlots) return comm_err("rt_frame_slot_wait: invalid argument", RT_ERR_INVALID_ARG);
    if (c->sent[slot] && hipStreamWaitEvent((hipStream_t)stream, c->gathered[slot], 0) != hipSuccess)
        return comm_err("rt_frame_slot_wait: stream ordering", RT_ERR_DEVICE);
    return RT_OK;
}

int rt_frame_ready_wait(rt_comm* c, int32_t slot, void* stream) {
    if (!c || slot < 0 || slot >= rt_comm::kSlots) return comm_err("rt_frame_ready_wait: invalid argument", RT_ERR_INVALID_ARG);
    hipEvent_t ev = c->rank == 0 ? c->assembled[slot] : c->gathered[slot];
    const bool done = c->rank == 0 ? c->built[slot] : c->sent[slot];
    if (done && hipStreamWaitEvent((hipStream_t)stream, ev, 0) != hipSuccess)
        return comm_err("rt_frame_ready_wait: stream ordering", RT_ERR_DEVICE);
    return RT_OK;
}

int rt_ipc_export(int32_t device, void* d_ptr, uint8_t* handle, int32_t handle_bytes, uint64_t* offset) {
    if (!d_ptr || !handle || !offset || handle_bytes < (int32_t)sizeof(hipIpcMemHandle_t))
        return comm_err("rt_ipc_export: invalid argument", RT_ERR_INVALID_ARG);
    if (hipSetDevice(device) != hipSuccess) return comm_err("rt_ipc_export: hipSetDevice", RT_ERR_DEVICE);
    // the handle names the whole allocation d_ptr lies in (a caching allocator's segment)
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d_ptr);
    if (e != hipSuccess) return comm_err(std::string("rt_ipc_export: hipMemGetAddressRange: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    hipIpcMemHandle_t h;
    if ((e = hipIpcGetMemHandle(&h, (void*)base)) != hipSuccess)
        return comm_err(std::string("rt_ipc_export: hipIpcGetMemHandle: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    std::memcpy(handle, &h, sizeof h);
    *offset = (uint64_t)((uintptr_t)d_ptr - (uintptr_t)base);
    return RT_OK;
}

int rt_ipc_open(int32_t device, const uint8_t* handle, int32_t handle_bytes, void** d_ptr) {
    if (!d_ptr || !handle || handle_bytes < (int32_t)sizeof(hipIpcMemHandle_t))
        return comm_err("rt_ipc_open: invalid argument", RT_ERR_INVALID_ARG);
    *d_ptr = nullptr;
    if (hipSetDevice(device) != hipSuccess) return comm_err("rt_ipc_open: hipSetDevice", RT_ERR_DEVICE);
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof h);
    const hipError_t e = hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        *d_ptr = nullptr;
        (void)hipGetLastError();   // the failure is reported here; later calls must not see it as theirs
        return comm_err(std::string("rt_ipc_open: hipIpcOpenMemHandle: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    }
    return RT_OK;
}

int rt_peer_access(int32_t device, int32_t peer, int32_t* can) {
    if (!can) return comm_err("rt_peer_access: invalid argument", RT_ERR_INVALID_ARG);
    *can = 0;
    if (device == peer) {   // the same GPU: its own memory
        *can = 1;
        return RT_OK;
    }
    int v = 0;
    const hipError_t e = hipDeviceCanAccessPeer(&v, device, peer);
    if (e != hipSuccess) return comm_err(std::string("rt_peer_access: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    *can = v ? 1 : 0;
    return RT_OK;
}

// Rank 0's shared frames + frame-sync block: written by other GPUs over xGMI while rank 0's
// kernels poll and read them, so not coarse-grained hipMalloc memory (coherent only at kernel
// boundaries) but uncached device memory (MTYPE UC: no L2 line can go stale on any GPU, the
// same kind RCCL uses for its cross-GPU flags and FIFOs).  Zeroed.
int rt_shared_alloc(int32_t device, uint64_t bytes, void** d_ptr) {
    if (!d_ptr || bytes == 0) return comm_err("rt_shared_alloc: invalid argument", RT_ERR_INVALID_ARG);
    *d_ptr = nullptr;
    if (hipSetDevice(device) != hipSuccess) return comm_err("rt_shared_alloc: hipSetDevice", RT_ERR_DEVICE);
    hipError_t e = hipExtMallocWithFlags(d_ptr, (size_t)bytes, hipDeviceMallocUncached);
    if (e != hipSuccess) {
        *d_ptr = nullptr;
        return comm_err(std::string("rt_shared_alloc: hipExtMallocWithFlags: ") + hipGetErrorString(e),
                        RT_ERR_OUT_OF_MEMORY);
    }
    if ((e = hipMemset(*d_ptr, 0, (size_t)bytes)) != hipSuccess) {
        (void)hipFree(*d_ptr);
        *d_ptr = nullptr;
        return comm_err(std::string("rt_shared_alloc: hipMemset: ") + hipGetErrorString(e), RT_ERR_DEVICE);
    }
    return RT_OK;
}

int rt_shared_free(int32_t device, void* d_ptr) {
    if (!d_ptr) return RT_OK;
    (void)hipSetDevice(device);
    return hipFree(d_ptr) == hipSuccess ? RT_OK : comm_err("rt_shared_free: hipFree", RT_ERR_DEVICE);
}

int rt_copy_device(void* d_dst, const void* d_src, uint64_t bytes, void* stream) {
    if ((!d_dst || !d_src) && bytes) return comm_err("rt_copy_device: invalid argument", RT_ERR_INVALID_ARG);
    const hipError_t e = hipMemcpyAsync(d_dst, d_src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    return e == hipSuccess ? RT_OK : comm_err(std::string("rt_copy_device: ") + hipGetErrorString(e), RT_ERR_DEVICE);
}

int rt_ipc_close(int32_t device, void* d_ptr) {
    if (!d_ptr) return RT_ERR_INVALID_ARG;
    (void)hipSetDevice(device);
    return hipIpcCloseMemHandle(d_ptr) == hipSuccess ? RT_OK : comm_err("rt_ipc_close: hipIpcCloseMemHandle", RT_ERR_DEVICE);
}

}  // extern "C"
