// pk_bisect_host.cpp -- diagnostic (never shipped): runs one victim kernel of a permlane_stress code
// object (tools/ubench/pk_bisect.py builds edited copies of its assembly) beside repeated launches of
// the MFMA aggressor, as permlane_stress's main() does, and prints the lane-disagreement counts.
// build: hipcc -O2 tools/ubench/pk_bisect_host.cpp -o tools/ubench/pk_bisect_host
// usage: pk_bisect_host CODE_OBJECT VICTIM_SYMBOL AGGRESSOR(0|1) ITERS
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s CODE_OBJECT VICTIM_SYMBOL AGGRESSOR(0|1) ITERS\n", argv[0]);
    return 2;
  }
  const int ak = atoi(argv[3]);
  int iters = atoi(argv[4]);
  hipModule_t mod;
  CK(hipModuleLoad(&mod, argv[1]));
  hipFunction_t fv, fa;
  CK(hipModuleGetFunction(&fv, mod, argv[2]));
  CK(hipModuleGetFunction(&fa, mod, "_Z9aggressorILi1EEviPf"));
  unsigned long long* d = nullptr;
  float* sink = nullptr;
  CK(hipMalloc(&d, 16));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(d, 0, 16));
  hipStream_t sv, sa;
  CK(hipStreamCreateWithFlags(&sv, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  hipEvent_t done;
  CK(hipEventCreate(&done));
  int aiters = 2000;
  void* aargs[] = {&aiters, &sink};
  auto launch_aggr = [&]() {
    return hipModuleLaunchKernel(fa, 2048, 1, 1, 256, 1, 1, 0, sa, aargs, nullptr);
  };
  if (ak)
    for (int k = 0; k < 4; ++k) CK(launch_aggr());  // aggressors first: the victim's blocks land among them
  unsigned long long* db = d;
  unsigned long long* dc = d + 1;
  void* vargs[] = {&iters, &db, &dc};
  CK(hipModuleLaunchKernel(fv, 256, 1, 1, 512, 1, 1, 0, sv, vargs, nullptr));
  CK(hipEventRecord(done, sv));
  int n_aggr = 4;
  while (ak && hipEventQuery(done) == hipErrorNotReady && n_aggr < 20000) {
    CK(launch_aggr());
    ++n_aggr;
    if (n_aggr % 8 == 0) CK(hipStreamSynchronize(sa));  // keep the queue short
  }
  CK(hipDeviceSynchronize());
  unsigned long long h[2];
  CK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
  printf("lanes0_47 %llu lanes48_63 %llu steps %llu aggressor_launches %d\n", h[0] & 0xFFFFFFFFull, h[0] >> 32, h[1],
         ak ? n_aggr : 0);
  CK(hipModuleUnload(mod));
  return 0;
}
