// Launch cost of an (almost) empty kernel vs grid size and LDS, replayed as a
// hipGraph of N dependent launches (what the cell's frame loop looks like).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void k_empty(int* flag) {
  extern __shared__ char smem[];
  if (threadIdx.x == 0 && blockIdx.x == 0 && flag[0] == 12345) smem[0] = 1, flag[1] = smem[0];
}

int main() {
  int* flag;
  hipMalloc(&flag, 64);
  hipMemset(flag, 0, 64);
  hipFuncSetAttribute((const void*)k_empty, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipStream_t st;
  hipStreamCreate(&st);
  const int N = 400;
  int grids[] = {256, 512, 1024, 2048, 4096};
  int ldss[] = {0, 64 * 1024, 120 * 1024};
  int blocks[] = {256, 512};
  for (int bl : blocks)
    for (int lds : ldss)
      for (int g : grids) {
        if (bl == 512 && lds > 80 * 1024) continue;
        hipGraph_t gr;
        hipGraphExec_t ge;
        hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
        for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(g), dim3(bl), lds, st, flag);
        hipStreamEndCapture(st, &gr);
        hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        hipGraphLaunch(ge, st);
        hipStreamSynchronize(st);
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventRecord(a, st);
        for (int r = 0; r < 5; ++r) hipGraphLaunch(ge, st);
        hipEventRecord(b, st);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("block %4d  lds %6d  grid %5d : %.2f us/launch\n", bl, lds, g, ms * 1e3 / (5 * N));
        hipGraphExecDestroy(ge);
        hipGraphDestroy(gr);
      }
  return 0;
}
