// Probe: does the raw-buffer range check include soffset on gfx950?  Descriptor over the
// first 4096 bytes of a 64 KiB buffer filled with 1.0f; loads at voffset 0 + soffset S and at
// voffset S + soffset 0.  A load past num_records reads 0, one inside reads 1.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(const float* buf, int soff, float* out) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, 0, 4096, 0x00020000);
    const int s = __builtin_amdgcn_readfirstlane(soff);
    out[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 0, s, 0));
    out[1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, s, 0, 0));
    out[2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 4092 - s, s, 0));
}

int main() {
    float *buf, *out;
    if (hipMalloc(&buf, 65536) != hipSuccess || hipMalloc(&out, 16) != hipSuccess) return 2;
    float h[16384];
    for (int i = 0; i < 16384; ++i) h[i] = 1.0f;
    hipMemcpy(buf, h, 65536, hipMemcpyHostToDevice);
    for (int soff : {0, 4092, 4096, 8192, 32768}) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, soff, out);
        float o[3];
        hipMemcpy(o, out, 12, hipMemcpyDeviceToHost);
        printf("soffset %6d: (v=0, s=S) -> %g   (v=S, s=0) -> %g   (v=4092-S, s=S) -> %g\n", soff, o[0], o[1], o[2]);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
