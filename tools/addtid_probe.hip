// addtid_probe.hip -- where does ds_write_addtid_b32 put each lane's dword?  (tools only)
// One 256-thread block: wave w sets M0 = 256 * w + 4096 * (w & 1) and stores tid + 1 at
// instruction offsets 0 and 32768; the LDS image is copied out and every written word is
// printed as (byte address, writer tid), so the address formula can be read off.  Result (r04l):
// address = M0[15:0] + offset + 4 * lane, provided the M0 write is followed by wait states (s_nop):
// without them the first store after s_mov m0 used the previous M0 (128 of 512 words lost).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) probe(uint32_t *out) {
    __shared__ uint32_t s[16384];
    for (int i = threadIdx.x; i < 16384; i += 256) s[i] = 0;
    __syncthreads();
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t b = __builtin_amdgcn_readfirstlane(256u * w + 4096u * (w & 1u));
    const uint32_t v = threadIdx.x + 1;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 1\n\tds_write_addtid_b32 %1\n\tds_write_addtid_b32 %1 offset:32768\n\ts_waitcnt lgkmcnt(0)"
                 :
                 : "s"(b), "v"(v)
                 : "memory", "m0");
#pragma clang diagnostic pop
    __syncthreads();
    for (int i = threadIdx.x; i < 16384; i += 256) out[i] = s[i];
}

int main() {
    uint32_t *d;
    if (hipMalloc(&d, 16384 * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, d);
    std::vector<uint32_t> h(16384);
    if (hipMemcpy(h.data(), d, 16384 * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int n = 0;
    for (int i = 0; i < 16384; ++i)
        if (h[i]) {
            const int tid = (int)h[i] - 1;
            if (tid % 16 == 0 || tid % 64 == 63) printf("byte %6d <- tid %3d (wave %d lane %2d)\n", 4 * i, tid, tid / 64, tid % 64);
            ++n;
        }
    printf("%d words written (expected 512)\n", n);
    return 0;
}
