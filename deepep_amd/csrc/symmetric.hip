// symmetric.hip -- the symmetric receive buffer over xGMI and its device barrier.
//
// Reference (paths in /root/reference):
//   NCCLSymmetricMemoryContext: one registered window per rank, every peer's window
//   load/store-addressable over NVLink            csrc/elastic/nccl.cu:62-153, buffer.hpp:181-208
//   gpu_barrier / nvlink_barrier_wo_local_sync:
//   per-rank signal slots written by every peer   deep_ep/include/deep_ep/common/comm.cuh:88-129, 208-264
//
// MI355X design: the window is one hipExtMallocWithFlags(hipDeviceMallocUncached) allocation per
// rank, exported with hipIpcGetMemHandle and opened by every peer with hipIpcOpenMemHandle; the
// fabric (xGMI) makes the peer's HBM load/store addressable from kernels.  Uncached (MTYPE UC)
// memory is used because a peer's stores land in this GPU's HBM behind its L2; nothing of the
// window should ever be cached; measured, one-XCD fences were not enough (below), so a publishing
// launch first writes back the L2 of every XCD and a barrier / wait ends by invalidating every
// XCD's L2 (writeback_all_xcds, invalidate_all_xcds).  Then thread s of the last workgroup publishes `epoch` into
// rank s's flag slot [rank] with a system-scope release store and waits, with a system-scope
// acquire load, until its own slot [s] reaches `epoch`.  Epochs only grow, so flags never need resetting;
// they are counted on the device, so the barriers replay correctly inside a captured HIP graph.
// A wall-clock timeout (the reference's num_gpu_timeout_secs, comm.cuh:30-54) sets bit 2 of the
// error flag and lets the kernel finish instead of trapping, so a lost peer never hangs the GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/deepep_amd.h"

extern "C" int deepep_amd_set_error(int code, const char* msg);
extern "C" void deepep_amd_register_budget(void* stream, int cus);

namespace {

int hip_fail(hipError_t e, const char* what) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    return deepep_amd_set_error(DEEPEP_ERR_HIP, buf);
}

// Epochs counted on the device (argument <= 0): the next epoch comes from this rank's own counter
// in its window header, so a captured HIP graph replays with fresh epochs.  Counter table: int64
// [3][kSlots] after the flag table -- row 0 = publishes per slot (barrier = slot 0, signals),
// row 1 = waits per slot, row 2 = workgroup arrivals of the publishing launches (below).  Only the
// launching kernel touches its counters (one stream-ordered kernel at a time per slot).
constexpr int kSlots = DEEPEP_SYM_FLAG_SLOTS;

// Every XCD takes part in a hand-off.  Publishing launches (barrier, signal) run kXcdGroups
// workgroups -- dealt round-robin over the 8 XCDs, so every XCD gets some: each writes back its
// XCD's L2 at system scope and waits for it, then counts its arrival, and the last to arrive
// publishes.  After a barrier or a wait, kXcdGroups workgroups invalidate every XCD's L2 before the
// stream's next kernel reads the window.  A single-workgroup fence covers one XCD only.  Evidence
// (tests/test_xgmi_gpu.py config 3 after the 8-process test, 8 processes sharing one GPU): with
// the one-XCD fences about one first dispatch / combine in five read stale rows; with the
// write-back alone 1 in 14; with write-back and invalidate 0 in 22, as with host-synchronised
// hand-offs (0 in 18).
constexpr int kXcdGroups = 64;

__device__ __forceinline__ bool writeback_all_xcds(const uint64_t* peer_flags, int rank, int slot) {
    __shared__ int s_last;
    if (threadIdx.x == 0) {
        // buffer_wbl2 sc0 sc1, then buffer_inv sc0 sc1: this XCD's dirty lines reach memory and its
        // copies of window lines are dropped, so the last workgroup reads its epoch counter fresh
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int64_t* join = reinterpret_cast<int64_t*>(peer_flags[rank]) + kSlots * 64 + 2 * kSlots + slot;
        const int64_t arrived = __hip_atomic_fetch_add(join, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
        s_last = arrived % static_cast<int64_t>(gridDim.x) == 0;
    }
    __syncthreads();
    return s_last != 0;
}

__device__ __forceinline__ int64_t next_epoch(const uint64_t* peer_flags, int rank, int row, int slot, int64_t given) {
    __shared__ int64_t s_epoch;
    if (threadIdx.x == 0) {
        int64_t e = given;
        if (e <= 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");             // no stale copy of the counter
            int64_t* cnt = reinterpret_cast<int64_t*>(peer_flags[rank]) + kSlots * 64 + row * kSlots + slot;
            e = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
            __hip_atomic_store(cnt, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_epoch = e;
    }
    __syncthreads();
    return s_epoch;
}

__device__ __forceinline__ void wait_slots(const int64_t* mine, int s, int64_t epoch, int64_t timeout_ticks,
                                           int32_t* error_flag) {
    // An acquire load invalidates this XCD's L2 only AFTER it has read: a stale copy of the flag line
    // left in that L2 (window memory freed by an earlier process and reallocated here still holds
    // that process's epochs) would let the very first poll pass early.  Drop such copies first.
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");                     // buffer_inv sc0 sc1
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(mine + s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
        if (static_cast<int64_t>(wall_clock64() - t0) > timeout_ticks) {
            if (error_flag != nullptr) atomicOr(error_flag, 2);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

__global__ void __launch_bounds__(64)
sym_barrier_kernel(const uint64_t* peer_flags, int rank, int num_ranks, int64_t epoch, int64_t timeout_ticks,
                   int32_t* error_flag) {
    if (!writeback_all_xcds(peer_flags, rank, 0)) return;
    epoch = next_epoch(peer_flags, rank, 0, 0, epoch);
    const int s = static_cast<int>(threadIdx.x);
    if (s >= num_ranks) return;
    __threadfence_system();
    int64_t* theirs = reinterpret_cast<int64_t*>(peer_flags[s]);
    __hip_atomic_store(theirs + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    wait_slots(reinterpret_cast<const int64_t*>(peer_flags[rank]), s, epoch, timeout_ticks, error_flag);
    __threadfence_system();
}

// Split barrier for pipelining: `signal` publishes `value` into slot `slot` of every rank's flag
// table (after this stream's earlier work), `wait` waits for every rank's signal in this rank's
// table.  Flag table of a window: int64 [kSlots][64], slot 0 is the full barrier above.
__global__ void __launch_bounds__(64)
sym_signal_kernel(const uint64_t* peer_flags, int rank, int num_ranks, int slot, int64_t value) {
    if (!writeback_all_xcds(peer_flags, rank, slot)) return;
    value = next_epoch(peer_flags, rank, 0, slot, value);
    const int s = static_cast<int>(threadIdx.x);
    if (s >= num_ranks) return;
    __threadfence_system();
    int64_t* theirs = reinterpret_cast<int64_t*>(peer_flags[s]) + static_cast<int64_t>(slot) * 64;
    __hip_atomic_store(theirs + rank, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(64)
sym_wait_kernel(const uint64_t* peer_flags, int rank, int num_ranks, int slot, int64_t value, int64_t timeout_ticks,
                int32_t* error_flag) {
    value = next_epoch(peer_flags, rank, 1, slot, value);
    const int s = static_cast<int>(threadIdx.x);
    if (s >= num_ranks) return;
    wait_slots(reinterpret_cast<const int64_t*>(peer_flags[rank]) + static_cast<int64_t>(slot) * 64, s, value,
               timeout_ticks, error_flag);
    __threadfence_system();
}

// The notify put: workgroup d copies src row d (bytes) into destination d's window at dest_offset with
// system-scope write-through stores (they reach the peer's HBM; the barrier after the put orders them).
__global__ void __launch_bounds__(256)
sym_put_kernel(const uint32_t* __restrict__ src, int64_t bytes, const uint64_t* __restrict__ dest_bases,
               int64_t dest_offset, const int32_t* __restrict__ error_flag) {
    if (error_flag != nullptr && (__hip_atomic_load(error_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 2))
        return;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const int64_t d = blockIdx.x;
    const u32x4* s = reinterpret_cast<const u32x4*>(src + d * (bytes / 4));
    uint8_t* dst = reinterpret_cast<uint8_t*>(dest_bases[d]) + dest_offset;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, static_cast<int>(bytes), 0x00020000);
    for (int64_t v = threadIdx.x; v < bytes / 16; v += blockDim.x)
        __builtin_amdgcn_raw_buffer_store_b128(s[v], rs, static_cast<int>(v * 16), 0, 17);    // sc0 sc1
}

// After a barrier or a wait: every XCD invalidates its L2 (system scope) before the stream's next
// kernel reads what the peers stored into this rank's window (one extra small launch).
__global__ void __launch_bounds__(64) invalidate_all_xcds_kernel() {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");                 // buffer_inv sc0 sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

hipError_t invalidate_all_xcds(hipStream_t s) {
    hipLaunchKernelGGL(invalidate_all_xcds_kernel, dim3(kXcdGroups), dim3(64), 0, s);
    return hipGetLastError();
}

int64_t timeout_ticks(int64_t timeout_us, int* rc) {
    static thread_local int64_t ticks_per_us = 0;
    *rc = DEEPEP_OK;
    if (ticks_per_us == 0) {
        int dev = 0, khz = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
        if (e != hipSuccess) {
            *rc = hip_fail(e, "wall clock rate");
            return 0;
        }
        ticks_per_us = khz > 1000 ? khz / 1000 : 1;
    }
    return (timeout_us > 0 ? timeout_us : 100000000LL) * ticks_per_us;
}

}  // namespace

extern "C" {

int deepep_sym_alloc(int64_t bytes, void** ptr) {
    if (ptr == nullptr || bytes <= 0) return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "sym_alloc: bad size");
    *ptr = nullptr;
    hipError_t e = hipExtMallocWithFlags(ptr, static_cast<size_t>(bytes), hipDeviceMallocUncached);
    if (e != hipSuccess) return hip_fail(e, "hipExtMallocWithFlags(uncached)");
    // Null-stream memset + null-stream sync (not a device-wide sync: ranks that share a process
    // may already have barrier kernels waiting on other streams).
    e = hipMemsetAsync(*ptr, 0, static_cast<size_t>(bytes), nullptr);
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) {
        (void)hipFree(*ptr);
        *ptr = nullptr;
        return hip_fail(e, "hipMemset(symmetric buffer)");
    }
    return DEEPEP_OK;
}

int deepep_sym_free(void* ptr) {
    if (ptr == nullptr) return DEEPEP_OK;
    const hipError_t e = hipFree(ptr);
    return e == hipSuccess ? DEEPEP_OK : hip_fail(e, "hipFree(symmetric buffer)");
}

int deepep_sym_export(void* ptr, void* handle) {
    static_assert(sizeof(hipIpcMemHandle_t) <= DEEPEP_IPC_HANDLE_BYTES, "IPC handle size");
    if (ptr == nullptr || handle == nullptr) return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "sym_export: null");
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, ptr);
    if (e != hipSuccess) return hip_fail(e, "hipIpcGetMemHandle");
    memset(handle, 0, DEEPEP_IPC_HANDLE_BYTES);
    memcpy(handle, &h, sizeof(h));
    return DEEPEP_OK;
}

int deepep_sym_import(const void* handle, void** ptr) {
    if (ptr == nullptr || handle == nullptr) return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "sym_import: null");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    *ptr = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
    return e == hipSuccess ? DEEPEP_OK : hip_fail(e, "hipIpcOpenMemHandle");
}

int deepep_sym_close(void* ptr) {
    if (ptr == nullptr) return DEEPEP_OK;
    const hipError_t e = hipIpcCloseMemHandle(ptr);
    return e == hipSuccess ? DEEPEP_OK : hip_fail(e, "hipIpcCloseMemHandle");
}

int deepep_stream_create_cu_budget(int num_cus, deepep_stream_t* stream) {
    if (stream == nullptr || num_cus < 1) return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "cu_budget: bad arguments");
    *stream = nullptr;
    int dev = 0, n = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return hip_fail(e, "CU count");
    // Mask bit b is CU b / 8 of XCD b % 8 (probed on MI355X, tools/probe_cumask.py), and an XCD whose
    // bits are all clear is not restricted at all; so the budget is the FIRST num_cus bits, rounded up
    // to a whole number of CUs per XCD (a multiple of 8, at least 8): fewer bits would leave whole XCDs
    // unrestricted, and a remainder would spread the budget unevenly.
    num_cus = (num_cus + 7) / 8 * 8;
    if (num_cus > n) num_cus = n;
    uint32_t mask[64] = {};
    const int words = (n + 31) / 32;
    if (words > 64) return deepep_amd_set_error(DEEPEP_ERR_UNSUPPORTED, "cu_budget: more than 2048 CUs");
    for (int b = 0; b < num_cus; ++b) mask[b / 32] |= 1u << (b % 32);
    hipStream_t s = nullptr;
    e = hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(words), mask);
    if (e != hipSuccess) return hip_fail(e, "hipExtStreamCreateWithCUMask");
    deepep_amd_register_budget(s, num_cus);          // combine launches on it cap rows in flight at 4
    *stream = reinterpret_cast<deepep_stream_t>(s);
    return DEEPEP_OK;
}

namespace {
// Where the workgroups of a stream run (diagnostic for CU budgets): HW_REG_HW_ID and HW_REG_XCC_ID of
// every workgroup's first lane.
__global__ void where_kernel(uint32_t* out, int spin) {
    if (threadIdx.x != 0) return;
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));
    for (volatile int i = 0; i < spin; ++i) {}
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
}
}  // namespace

int deepep_stream_probe_cus(deepep_stream_t stream, int* num_cus, int* num_xcds) {
    if (num_cus == nullptr || num_xcds == nullptr) return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "probe_cus: null");
    constexpr int kBlocks = 8192;
    uint32_t* d = nullptr;
    hipError_t e = hipMalloc(&d, sizeof(uint32_t) * 2 * kBlocks);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(probe)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(where_kernel, dim3(kBlocks), dim3(64), 0, s, d, 2000);
    static uint32_t h[2 * kBlocks];
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "probe_cus");
    bool seen[16][8][2][16] = {};            // (xcc, se, sh, cu)
    bool xcds[16] = {};
    int n = 0, x = 0;
    for (int i = 0; i < kBlocks; ++i) {
        const uint32_t hw = h[2 * i], xcc = h[2 * i + 1] & 0xF;
        const uint32_t cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 0x1, se = (hw >> 13) & 0x7;
        if (!seen[xcc][se][sh][cu]) { seen[xcc][se][sh][cu] = true; ++n; }
        if (!xcds[xcc]) { xcds[xcc] = true; ++x; }
    }
    *num_cus = n;
    *num_xcds = x;
    return DEEPEP_OK;
}

int deepep_stream_destroy(deepep_stream_t stream) {
    if (stream == nullptr) return DEEPEP_OK;
    deepep_amd_register_budget(stream, 0);
    const hipError_t e = hipStreamDestroy(reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? DEEPEP_OK : hip_fail(e, "hipStreamDestroy");
}

int deepep_sym_put(const void* src, int64_t bytes, const uint64_t* dest_bases, int num_ranks, int64_t dest_offset,
                   int64_t dest_extent, const int32_t* error_flag, deepep_stream_t stream) {
    if (num_ranks < 1 || num_ranks > 64 || bytes < 0 || bytes % 16 || bytes > (int64_t(1) << 30) || dest_offset < 0 ||
        dest_offset % 16 || (bytes > 0 && (src == nullptr || dest_bases == nullptr)) ||
        (reinterpret_cast<uintptr_t>(src) & 15))
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "sym_put: bad arguments");
    // every store lands in [dest_bases[d] + dest_offset, + bytes): it must lie inside the destination's
    // window (dest_extent bytes from its base), whatever the caller computed
    if (dest_extent < 0 || dest_offset > dest_extent || bytes > dest_extent - dest_offset)
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "sym_put: [dest_offset, dest_offset + bytes) lies outside "
                                                            "the destination window (dest_extent)");
    if (bytes == 0) return DEEPEP_OK;
    hipLaunchKernelGGL(sym_put_kernel, dim3(num_ranks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       static_cast<const uint32_t*>(src), bytes, dest_bases, dest_offset, error_flag);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DEEPEP_OK : hip_fail(e, "put launch");
}

int deepep_sym_barrier(const uint64_t* peer_flags, int rank, int num_ranks, int64_t epoch, int64_t timeout_us,
                       int32_t* error_flag, deepep_stream_t stream) {
    if (peer_flags == nullptr || num_ranks < 1 || num_ranks > 64 || rank < 0 || rank >= num_ranks)
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "sym_barrier: bad arguments");
    int rc = DEEPEP_OK;
    const int64_t ticks = timeout_ticks(timeout_us, &rc);
    if (rc != DEEPEP_OK) return rc;
    hipLaunchKernelGGL(sym_barrier_kernel, dim3(kXcdGroups), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                       peer_flags, rank, num_ranks, epoch, ticks, error_flag);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = invalidate_all_xcds(reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? DEEPEP_OK : hip_fail(e, "barrier launch");
}

int deepep_sym_signal(const uint64_t* peer_flags, int rank, int num_ranks, int slot, int64_t value,
                      deepep_stream_t stream) {
    if (peer_flags == nullptr || num_ranks < 1 || num_ranks > 64 || rank < 0 || rank >= num_ranks || slot < 1 ||
        slot >= DEEPEP_SYM_FLAG_SLOTS)
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "sym_signal: bad arguments");
    hipLaunchKernelGGL(sym_signal_kernel, dim3(kXcdGroups), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                       peer_flags, rank, num_ranks, slot, value);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DEEPEP_OK : hip_fail(e, "signal launch");
}

int deepep_sym_wait(const uint64_t* peer_flags, int rank, int num_ranks, int slot, int64_t value, int64_t timeout_us,
                    int32_t* error_flag, deepep_stream_t stream) {
    if (peer_flags == nullptr || num_ranks < 1 || num_ranks > 64 || rank < 0 || rank >= num_ranks || slot < 1 ||
        slot >= DEEPEP_SYM_FLAG_SLOTS)
        return deepep_amd_set_error(DEEPEP_ERR_INVALID_ARG, "sym_wait: bad arguments");
    int rc = DEEPEP_OK;
    const int64_t ticks = timeout_ticks(timeout_us, &rc);
    if (rc != DEEPEP_OK) return rc;
    hipLaunchKernelGGL(sym_wait_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                       peer_flags, rank, num_ranks, slot, value, ticks, error_flag);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = invalidate_all_xcds(reinterpret_cast<hipStream_t>(stream));
    return e == hipSuccess ? DEEPEP_OK : hip_fail(e, "wait launch");
}

}  // extern "C"
