// Does the raw-buffer range check include the instruction's scalar offset (soffset)?  (tools only)
// A 4 KB allocation filled with 1.0f, a descriptor over its first 256 bytes; lane 0 loads with
// (voffset, soffset) = (0, 512) and (512, 0) and stores with (0, 512).  Every access stays inside
// the allocation, so either answer is safe to observe.
//   hipcc --offload-arch=gfx950 -O2 -o tools/_build/soffset_probe tools/soffset_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void probe(float* buf, float* out) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, 256, 0x00020000);
    if (threadIdx.x == 0) {
        int so = 512;
        asm volatile("" : "+s"(so));
        out[0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 0, so, 0));
        out[1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 512, 0, 0));
        out[2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, 7.0f), r, 0, so + 4, 0);
    }
}

int main() {
    float *buf, *out;
    if (hipMalloc(&buf, 4096) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    float h[1024];
    for (auto& v : h) v = 1.0f;
    hipMemcpy(buf, h, 4096, hipMemcpyHostToDevice);
    hipMemset(out, 0xff, 64);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, out);
    float o[3];
    hipMemcpy(o, out, 12, hipMemcpyDeviceToHost);
    hipMemcpy(h, buf, 4096, hipMemcpyDeviceToHost);
    std::printf("load (v=0, s=512): %g  load (v=512, s=0): %g  load (0, 0): %g  store (v=0, s=516) landed: %s\n", o[0], o[1],
                o[2], h[129] == 7.0f ? "yes" : "no");
    std::printf("soffset %s in the range check\n", (o[0] == 0.0f && h[129] != 7.0f) ? "IS" : "is NOT");
    return 0;
}
