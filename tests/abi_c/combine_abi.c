/* combine_abi.c -- a plain C consumer of the C-ABI (include/deepep_amd.h): no Python, no torch.
 *
 * What a host runtime binding the library from C (or cgo / any FFI) does for the EP = 1 combine:
 * hipMalloc the expanded expert rows, the handle's recv_src_metadata and the outputs, turn the
 * metadata into the token-major slot plan (deepep_build_local_plan), run the fused reduction
 * (deepep_combine_reduce, MODE_FUSED: plain + bias, gating-weighted, weight pass-through) and
 * check every output bit against the CPU oracle (oracle/combine_ref.c, linked as the checker).
 * Also checks that invalid arguments come back as DEEPEP_ERR_INVALID_ARG with a message.
 * Test infrastructure: built by __graft_entry__.build(), run by tests/test_abi_c_gpu.py. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/deepep_amd.h"

int oracle_combine_rows(int mode, int weighted, const uint16_t* src, int64_t num_src_rows, int64_t src_stride,
                        const int32_t* table, int64_t table_stride, int table_width, const float* row_weights,
                        const uint16_t* bias0, const uint16_t* bias1, uint16_t* out, int64_t out_stride,
                        int num_units, int hidden, const int32_t* wtable, int64_t wtable_stride, const float* wsrc,
                        float* out_weights, int num_weights, int64_t out_weights_stride);

static uint64_t g_state = 0x9e3779b97f4a7c15ull;
static uint32_t rnd(void) {
    g_state ^= g_state << 13;
    g_state ^= g_state >> 7;
    g_state ^= g_state << 17;
    return (uint32_t)(g_state >> 16);
}
static uint16_t rnd_bf16(void) {            /* a normal-range bf16: sign, exponent 120..134, mantissa */
    return (uint16_t)(((rnd() & 1u) << 15) | ((120u + rnd() % 15u) << 7) | (rnd() & 0x7fu));
}

#define CHECK_HIP(e) do { hipError_t _e = (e); if (_e != hipSuccess) { \
    fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(_e), __LINE__); return 2; } } while (0)
#define CHECK_EP(e) do { int _r = (e); if (_r != DEEPEP_OK) { \
    fprintf(stderr, "deepep error %d (%s) at line %d\n", _r, deepep_amd_last_error(), __LINE__); return 3; } } while (0)

int main(void) {
    const int T = 300, H = 2048, K = 8;
    const int64_t N = (int64_t)T * K;                      /* expanded rows */
    if (deepep_amd_abi_version() != DEEPEP_AMD_ABI_VERSION) {
        fprintf(stderr, "ABI %d != header %d\n", deepep_amd_abi_version(), DEEPEP_AMD_ABI_VERSION);
        return 4;
    }
    uint16_t* y = malloc(N * H * 2);
    uint16_t* bias = malloc((size_t)T * H * 2);
    float* w = malloc(N * 4);
    int32_t* meta = malloc((size_t)T * (K + 2) * 4);
    int32_t* table = malloc((size_t)T * K * 4);
    int32_t* plan = malloc((size_t)T * K * 4);
    int64_t* perm = malloc(N * 8);
    uint16_t *got = malloc((size_t)T * H * 2), *want = malloc((size_t)T * H * 2);
    float *got_w = malloc((size_t)T * K * 4), *want_w = malloc((size_t)T * K * 4);
    for (int64_t i = 0; i < N * H; ++i) y[i] = rnd_bf16();
    for (int64_t i = 0; i < (int64_t)T * H; ++i) bias[i] = rnd_bf16();
    for (int64_t i = 0; i < N; ++i) w[i] = (float)(rnd() % 1000000) / 1e6f;
    for (int64_t i = 0; i < N; ++i) perm[i] = i;
    for (int64_t i = N - 1; i > 0; --i) {                  /* expanded rows in a random order */
        const int64_t j = rnd() % (i + 1), tmp = perm[i];
        perm[i] = perm[j], perm[j] = tmp;
    }
    for (int t = 0; t < T; ++t) {
        int master = 0;
        for (int k = 0; k < K; ++k) {
            const int valid = (rnd() % 10) != 0 || k == 0;  /* ~10 % masked top-k slots */
            table[t * K + k] = valid ? (int32_t)perm[t * K + k] : -1;
            if (valid) master = k;
        }
        meta[t * (K + 2) + 0] = t;                         /* src_rank 0 * T_max + t */
        meta[t * (K + 2) + 1] = master;
        for (int k = 0; k < K; ++k) meta[t * (K + 2) + 2 + k] = table[t * K + k];
    }

    void *d_y, *d_bias, *d_w, *d_meta, *d_plan, *d_out, *d_out_w, *d_err;
    CHECK_HIP(hipMalloc(&d_y, N * H * 2));
    CHECK_HIP(hipMalloc(&d_bias, (size_t)T * H * 2));
    CHECK_HIP(hipMalloc(&d_w, N * 4));
    CHECK_HIP(hipMalloc(&d_meta, (size_t)T * (K + 2) * 4));
    CHECK_HIP(hipMalloc(&d_plan, (size_t)T * K * 4));
    CHECK_HIP(hipMalloc(&d_out, (size_t)T * H * 2));
    CHECK_HIP(hipMalloc(&d_out_w, (size_t)T * K * 4));
    CHECK_HIP(hipMalloc(&d_err, 4));
    CHECK_HIP(hipMemcpy(d_y, y, N * H * 2, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d_bias, bias, (size_t)T * H * 2, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d_w, w, N * 4, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(d_meta, meta, (size_t)T * (K + 2) * 4, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemset(d_err, 0, 4));

    /* the handle's metadata -> token-major slot plan */
    CHECK_EP(deepep_build_local_plan(d_meta, T, K, T, 1, d_plan, K, T, NULL, NULL, NULL));
    CHECK_HIP(hipMemcpy(plan, d_plan, (size_t)T * K * 4, hipMemcpyDeviceToHost));
    int fails = 0;
    if (memcmp(plan, table, (size_t)T * K * 4) != 0) {
        fprintf(stderr, "build_local_plan: plan differs from the metadata slots\n");
        ++fails;
    }

    for (int weighted = 0; weighted <= 1; ++weighted)
        for (int with_bias = 0; with_bias <= 1; ++with_bias) {
            const void* b0 = with_bias ? d_bias : NULL;
            CHECK_EP(deepep_combine_reduce(DEEPEP_MODE_FUSED, weighted, d_y, N, H, d_plan, K, K, weighted ? d_w : NULL,
                                           b0, NULL, d_out, H, T, H, d_plan, K, d_w, d_out_w, K, 0, 0, 0, d_err, NULL));
            CHECK_HIP(hipDeviceSynchronize());
            CHECK_HIP(hipMemcpy(got, d_out, (size_t)T * H * 2, hipMemcpyDeviceToHost));
            CHECK_HIP(hipMemcpy(got_w, d_out_w, (size_t)T * K * 4, hipMemcpyDeviceToHost));
            if (oracle_combine_rows(DEEPEP_MODE_FUSED, weighted, y, N, H, table, K, K, weighted ? w : NULL,
                                    with_bias ? bias : NULL, NULL, want, H, T, H, table, K, w, want_w, K, 0) != 0) {
                fprintf(stderr, "oracle rejected the case\n");
                return 5;
            }
            const int ok_x = memcmp(got, want, (size_t)T * H * 2) == 0;
            const int ok_w = memcmp(got_w, want_w, (size_t)T * K * 4) == 0;
            printf("fused weighted=%d bias=%d: combined_x %s, combined_topk_weights %s\n", weighted, with_bias,
                   ok_x ? "bitwise equal" : "DIFFERS", ok_w ? "bitwise equal" : "DIFFERS");
            fails += !ok_x + !ok_w;
        }
    int32_t err_flag = -1;
    CHECK_HIP(hipMemcpy(&err_flag, d_err, 4, hipMemcpyDeviceToHost));
    if (err_flag != 0) {
        fprintf(stderr, "error flag %d set on in-range slots\n", err_flag);
        ++fails;
    }
    /* error convention: hidden % 8 != 0 is rejected on the host, with a message, nothing launched */
    const int rc = deepep_combine_reduce(DEEPEP_MODE_FUSED, 0, d_y, N, H, d_plan, K, K, NULL, NULL, NULL, d_out, H, T,
                                         H - 4, NULL, 0, NULL, NULL, 0, 0, 0, 0, NULL, NULL);
    if (rc != DEEPEP_ERR_INVALID_ARG || strlen(deepep_amd_last_error()) == 0) {
        fprintf(stderr, "invalid hidden: rc %d, message '%s'\n", rc, deepep_amd_last_error());
        ++fails;
    } else {
        printf("invalid hidden rejected: %s\n", deepep_amd_last_error());
    }
    hipFree(d_y), hipFree(d_bias), hipFree(d_w), hipFree(d_meta), hipFree(d_plan);
    hipFree(d_out), hipFree(d_out_w), hipFree(d_err);
    free(y), free(bias), free(w), free(meta), free(table), free(plan), free(perm);
    free(got), free(want), free(got_w), free(want_w);
    printf(fails ? "FAIL (%d)\n" : "PASS\n", fails);
    return fails ? 1 : 0;
}
