// Prediction text on the GPU: binary32 -> Java Float.toString text, one thread per value.
//
// The reference's bolt serializes every softmax row with Jackson (InferenceBolt.java:88-90,
// PredObj.java:9), i.e. Float.toString per probability. On the host that is ~0.7 us per
// CIFAR image (10 values: std::to_chars + Java layout, codec::format_float_java), one core per
// 1.5 M images/s. Here the replica's stream formats the rows right after the softmax, and the
// host only concatenates fixed 16-byte slots (codec::encode_predictions_text).
//
// Digits follow the JDK 19+ specification (the one codec::format_float_java implements):
//   R = decimals that round to v (round half even), m = min length over R; T = decimals of R
//   of length m (of length 2 when m = 1); the result is the member of T closest to v (even
//   last digit on a tie).
// A p-digit candidate is floor or ceil of v * 10^q, q = p - 1 - floor(log10 v); membership in
// R and every rounding decision are exact comparisons of d * 10^-q against K * 2^E
// (exact_decimal.cuh), so no step relies on floating-point rounding. Membership is monotone in
// p, so m is found by bisection over p in [1, 9] (9 digits always round-trip a binary32).
// Layout (FloatingDecimal): 10^-3 <= |v| < 10^7 as plain decimal with at least one fraction
// digit, otherwise d.dddE<exp>. Slot: up to 15 characters, length in byte 15.
#include "common.cuh"
#include "gale/kernels.h"
#include "java_float.cuh"

namespace gale {
namespace {

__global__ __launch_bounds__(256) void format_floats_kernel(int n, const int* d_count, int per,
                                                            const float* __restrict__ x,
                                                            uint4* __restrict__ out,
                                                            const int* d_nrec, int* status,
                                                            int* status_out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (d_nrec && i < *d_nrec) {  // the parse verdicts: to the host, cleared for the next batch
    status_out[i] = status[i];
    status[i] = 0;
  }
  if (d_count) n = min(n, *d_count * per);
  if (i >= n) return;
  out[i] = java_float_slot(x[i]);  // one 16-byte store per value
}

}  // namespace

hipError_t format_floats_java(int n, const float* x, void* out16, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(format_floats_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     stream, n, nullptr, 1, x, static_cast<uint4*>(out16), nullptr, nullptr,
                     nullptr);
  return hipGetLastError();
}

hipError_t format_floats_java_dev(int max_n, const int* d_count, int per, const float* x,
                                  void* out16, hipStream_t stream) {
  if (max_n <= 0) return hipSuccess;
  hipLaunchKernelGGL(format_floats_kernel, dim3((unsigned)((max_n + 255) / 256)), dim3(256), 0,
                     stream, max_n, d_count, per, x, static_cast<uint4*>(out16), nullptr, nullptr,
                     nullptr);
  return hipGetLastError();
}

hipError_t format_floats_java_step(int max_n, const int* d_count, int per, const float* x,
                                   void* out16, const int* d_nrec, int* status, int* status_out,
                                   hipStream_t stream) {
  if (max_n <= 0) return hipSuccess;
  if (!d_nrec || !status || !status_out) return hipErrorInvalidValue;
  hipLaunchKernelGGL(format_floats_kernel, dim3((unsigned)((max_n + 255) / 256)), dim3(256), 0,
                     stream, max_n, d_count, per, x, static_cast<uint4*>(out16), d_nrec, status,
                     status_out);
  return hipGetLastError();
}

}  // namespace gale
