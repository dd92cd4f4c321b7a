#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
__global__ void k(const float* in, float* out) {
  float r = in[threadIdx.x];
  float c = 1.0e30f;
  float o;
  asm volatile("v_min_f32 %0, %1, %2" : "=v"(o) : "v"(r), "v"(c));
  out[threadIdx.x] = o;
  float m;
  asm volatile("v_max_f32 %0, 0, %1" : "=v"(m) : "v"(r));
  out[64 + threadIdx.x] = m;
  float lo = -1.0e30f, md;
  asm volatile("v_med3_f32 %0, %1, %2, %3" : "=v"(md) : "v"(r), "v"(lo), "v"(c));
  out[128 + threadIdx.x] = md;
}
int main() {
  float h[64] = {0};
  h[0] = NAN; h[1] = INFINITY - INFINITY; h[2] = -INFINITY; h[3] = INFINITY; h[4] = 2.0f; h[5] = -3.0f; h[6] = 2e30f;
  float *d, *o; hipMalloc(&d, 256); hipMalloc(&o, 768);
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o);
  float r[192]; hipMemcpy(r, o, 768, hipMemcpyDeviceToHost);
  for (int i = 0; i < 7; ++i) printf("in %g -> min %g  max0 %g  med3 %g\n", h[i], r[i], r[64 + i], r[128 + i]);
  return 0;
}
