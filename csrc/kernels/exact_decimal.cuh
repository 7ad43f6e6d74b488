// Exact decimal <-> binary arithmetic shared by the JSON parser (decimal -> binary32,
// json_parse.hip) and the prediction formatter (binary32 -> shortest decimal, format.hip):
// w * 10^q against K * 2^E compared exactly as 256-bit integers (w * 5^|q| from a table of
// 5^0..5^66, both sides left-aligned).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace gale {
namespace {

__constant__ uint64_t kPow5[67][3] = {
    {0x0000000000000001ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0000000000000005ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0000000000000019ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000000000000007dull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0000000000000271ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0000000000000c35ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0000000000003d09ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000000000001312dull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000000000005f5e1ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x00000000001dcd65ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x00000000009502f9ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0000000002e90eddull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000000000e8d4a51ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0000000048c27395ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000000016bcc41e9ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000000071afd498dull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0000002386f26fc1ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000000b1a2bc2ec5ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000003782dace9d9ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x00001158e460913dull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000056bc75e2d631ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0001b1ae4d6e2ef5ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x000878678326eac9ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x002a5a058fc295edull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x00d3c21bcecceda1ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x0422ca8b0a00a425ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x14adf4b7320334b9ull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x6765c793fa10079dull, 0x0000000000000000ull, 0x0000000000000000ull},
    {0x04fce5e3e2502611ull, 0x0000000000000002ull, 0x0000000000000000ull},
    {0x18f07d736b90be55ull, 0x000000000000000aull, 0x0000000000000000ull},
    {0x7cb2734119d3b7a9ull, 0x0000000000000032ull, 0x0000000000000000ull},
    {0x6f7c40458122964dull, 0x00000000000000fcull, 0x0000000000000000ull},
    {0x2d6d415b85acef81ull, 0x00000000000004eeull, 0x0000000000000000ull},
    {0xe32246c99c60ad85ull, 0x00000000000018a6ull, 0x0000000000000000ull},
    {0x6fab61f00de36399ull, 0x0000000000007b42ull, 0x0000000000000000ull},
    {0x2e58e9b04570f1fdull, 0x000000000002684cull, 0x0000000000000000ull},
    {0xe7bc90715b34b9f1ull, 0x00000000000c097cull, 0x0000000000000000ull},
    {0x86aed236c807a1b5ull, 0x00000000003c2f70ull, 0x0000000000000000ull},
    {0xa16a1b11e8262889ull, 0x00000000012ced32ull, 0x0000000000000000ull},
    {0x2712875988becaadull, 0x0000000005e0a1fdull, 0x0000000000000000ull},
    {0xc35ca4bfabb9f561ull, 0x000000001d6329f1ull, 0x0000000000000000ull},
    {0xd0cf37be5aa1cae5ull, 0x0000000092efd1b8ull, 0x0000000000000000ull},
    {0x140c16b7c528f679ull, 0x00000002deaf189cull, 0x0000000000000000ull},
    {0x643c7196d9ccd05dull, 0x0000000e596b7b0cull, 0x0000000000000000ull},
    {0xf52e37f2410011d1ull, 0x00000047bf19673dull, 0x0000000000000000ull},
    {0xc9e717bb45005915ull, 0x00000166bb7f0435ull, 0x0000000000000000ull},
    {0xf18376a85901bd69ull, 0x00000701a97b150cull, 0x0000000000000000ull},
    {0xb7915149bd08b30dull, 0x000023084f676940ull, 0x0000000000000000ull},
    {0x95d69670b12b7f41ull, 0x0000af298d050e43ull, 0x0000000000000000ull},
    {0xed30f03375d97c45ull, 0x00036bcfc1194751ull, 0x0000000000000000ull},
    {0xa1f4b1014d3f6d59ull, 0x00111b0ec57e6499ull, 0x0000000000000000ull},
    {0x29c77506823d22bdull, 0x00558749db77f700ull, 0x0000000000000000ull},
    {0xd0e549208b31adb1ull, 0x01aba4714957d300ull, 0x0000000000000000ull},
    {0x147a6da2b7f86475ull, 0x085a36366eb71f04ull, 0x0000000000000000ull},
    {0x6664242d97d9f649ull, 0x29c30f1029939b14ull, 0x0000000000000000ull},
    {0xfff4b4e3f741cf6dull, 0xd0cf4b50cfe20765ull, 0x0000000000000000ull},
    {0xffc78873d4490d21ull, 0x140c78940f6a24fdull, 0x0000000000000004ull},
    {0xfee5aa43256d41a5ull, 0x643e5ae44d12b8f5ull, 0x0000000000000014ull},
    {0xfa7c534fbb224839ull, 0xf537c675815d9ccdull, 0x0000000000000065ull},
    {0xe46da08ea7ab691dull, 0xca16e04b86d41005ull, 0x00000000000001fdull},
    {0x762422c946590d91ull, 0xf2726179a224501dull, 0x00000000000009f4ull},
    {0x4eb4adee5fbd43d5ull, 0xbc3be7602ab59093ull, 0x00000000000031c8ull},
    {0x898765a7deb25329ull, 0xad2b84e0d58bd2e0ull, 0x000000000000f8ebull},
    {0xafa4fc47597b9fcdull, 0x61d998642bbb1e62ull, 0x000000000004dc9aull},
    {0x6e38ed64bf6a1f01ull, 0xe93ff9f4daa797edull, 0x0000000000184f03ull},
    {0x271ca2f7bd129b05ull, 0x8e3fe1c84545f7a3ull, 0x0000000000798b13ull},
    {0xc38f2ed6b15d0719ull, 0xc73f68e95a5dd62full, 0x00000000025fb761ull},
};

struct U256 {
  uint64_t v[4];  // little-endian limbs
};

__device__ __forceinline__ U256 mul_u64_pow5(uint64_t a, int n) {
  U256 r;
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint64_t b = kPow5[n][i];
    const uint64_t lo = a * b, hi = __umul64hi(a, b);
    r.v[i] = lo + carry;
    carry = hi + (r.v[i] < lo ? 1u : 0u);
  }
  r.v[3] = carry;
  return r;
}

__device__ __forceinline__ int bitlen(const U256& x) {
  for (int i = 3; i >= 0; --i)
    if (x.v[i]) return 64 * i + 64 - __clzll((long long)x.v[i]);
  return 0;
}

__device__ __forceinline__ U256 shl(const U256& x, int s) {  // 0 <= s < 256
  U256 r = {{0, 0, 0, 0}};
  const int q = s >> 6, b = s & 63;
  for (int i = 3; i >= q; --i) {
    uint64_t v = x.v[i - q] << b;
    if (b && i - q - 1 >= 0) v |= x.v[i - q - 1] >> (64 - b);
    r.v[i] = v;
  }
  return r;
}

// sign of (w * 10^q) - (K * 2^E)
__device__ int cmp_decimal_dyadic(uint64_t w, int q, uint64_t K, int E) {
  U256 A, B;
  int sa, sb;
  if (q >= 0) {
    A = mul_u64_pow5(w, q);
    sa = q;
    B = {{K, 0, 0, 0}};
    sb = E;
  } else {
    A = {{w, 0, 0, 0}};
    sa = q;
    B = mul_u64_pow5(K, -q);
    sb = E;
  }
  const int la = bitlen(A), lb = bitlen(B);
  if (la + sa != lb + sb) return la + sa > lb + sb ? 1 : -1;
  A = shl(A, 256 - la);  // left-align: equal magnitudes of the leading bit
  B = shl(B, 256 - lb);
  for (int i = 3; i >= 0; --i)
    if (A.v[i] != B.v[i]) return A.v[i] > B.v[i] ? 1 : -1;
  return 0;
}

}  // namespace
}  // namespace gale
