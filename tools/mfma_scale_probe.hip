// Probe of v_mfma_scale_f32_16x16x128_f8f6f4 on gfx950 with e4m3 operands:
// (1) the A/B lane->k map, found with one-hot A fragments against a B whose
//     bytes encode their own (lane group, byte) position;
// (2) the meaning of the E8M0 scale operand (0, 127, 128, runtime vs literal),
//     checked on small-integer data against a host product.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_scale_probe.hip -o tools/mfma_scale_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

// block b: A one-hot at (lane b/32, byte b%32) = 1.0; B lane l byte j = code (l>>4, j)
__global__ void probe_map(const uint8_t* bcode, float* out) {
  int l = threadIdx.x, b = blockIdx.x;
  uint8_t a[32], bb[32];
  for (int j = 0; j < 32; ++j) {
    a[j] = (l == b / 32 && j == b % 32) ? 0x38 : 0;  // e4m3fn 1.0
    bb[j] = bcode[(l >> 4) * 32 + j];
  }
  v8i av, bv;
  memcpy(&av, a, 32);
  memcpy(&bv, bb, 32);
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) out[b * 256 + ((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

template <int MODE>
__global__ void probe_scale(const uint8_t* A, const uint8_t* B, int sa, int sb, float* out) {
  int l = threadIdx.x;
  v8i av, bv;
  memcpy(&av, A + l * 32, 32);
  memcpy(&bv, B + l * 32, 32);
  v4f c = {0, 0, 0, 0};
  if (MODE == 0) c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 0, 0, 0);
  if (MODE == 1) c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 127, 0, 127);
  if (MODE == 2) c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, sa, 0, sb);
  if (MODE == 3) c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 1, sa, 2, sb);
  for (int r = 0; r < 4; ++r) out[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

static float e4m3(uint8_t v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float f = e ? std::ldexp(1.f + m / 8.f, e - 7) : std::ldexp(m / 8.f, -6);
  if ((v & 0x7f) == 0x7f) f = NAN;
  return s ? -f : f;
}

int main() {
  // ---- (1) lane map ----
  uint8_t code[128];
  for (int c = 0; c < 128; ++c) code[c] = c < 126 ? (uint8_t)(c + 1) : (uint8_t)(0x81 + (c - 126));
  uint8_t* dcode; float* dmap;
  CK(hipMalloc(&dcode, 128));
  CK(hipMalloc(&dmap, 2048 * 256 * 4));
  CK(hipMemcpy(dcode, code, 128, hipMemcpyHostToDevice));
  probe_map<<<2048, 64>>>(dcode, dmap);
  CK(hipDeviceSynchronize());
  std::vector<float> m(2048 * 256);
  CK(hipMemcpy(m.data(), dmap, m.size() * 4, hipMemcpyDeviceToHost));
  // for each one-hot (lane L, byte J): which row is nonzero, and which B code it picked
  int h1 = 0, h2 = 0, bad = 0;
  for (int b = 0; b < 2048; ++b) {
    int L = b / 32, J = b % 32, row = -1, kc = -1, nz = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        float v = m[b * 256 + i * 16 + j];
        if (v != 0.f) {
          ++nz;
          if (row < 0) {
            row = i;
            for (int c = 0; c < 128; ++c) if (e4m3(code[c]) == v) kc = c;
          }
        }
      }
    // B code kc = (group g, byte jb) -> B holds k at that position; the A one-hot's k equals it
    int g = kc / 32, jb = kc % 32;
    int kA1 = 32 * (L >> 4) + J, kB1 = 32 * g + jb;  // H1: 32 consecutive k per lane group
    int kA2 = (J < 16 ? 16 * (L >> 4) + J : 64 + 16 * (L >> 4) + J - 16);
    int kB2 = (jb < 16 ? 16 * g + jb : 64 + 16 * g + jb - 16);
    if (row != (L & 15) || nz != 16) ++bad;
    if (kA1 == kB1) ++h1;
    if (kA2 == kB2) ++h2;
    if (b < 40 || (b % 97) == 0) printf("A lane %2d byte %2d -> row %2d nz %3d  B group %d byte %2d\n", L, J, row, nz, g, jb);
  }
  printf("map: row/nz mismatches %d; same-position(A,B) %d/2048\n", bad, h1);
  (void)h2;
  // ---- (2) scale semantics on integer data, assuming A lane l byte j = A[l&15][32(l>>4)+j] ----
  std::vector<uint8_t> A(64 * 32), B(64 * 32);
  std::vector<float> Af(16 * 128), Bf(128 * 16);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1103515245u + 12345u; return (s >> 16) & 0x7fff; };
  const uint8_t vals[9] = {0xC8, 0xC0, 0xB8, 0xB0, 0x00, 0x30, 0x38, 0x40, 0x48};  // -4,-2,-1,-0.5,0,.5,1,2,4
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 32; ++j) {
      uint8_t a = vals[rnd() % 9], b = vals[rnd() % 9];
      A[l * 32 + j] = a; B[l * 32 + j] = b;
      Af[(l & 15) * 128 + 32 * (l >> 4) + j] = e4m3(a);
      Bf[(32 * (l >> 4) + j) * 16 + (l & 15)] = e4m3(b);
    }
  std::vector<double> ref(256, 0.0);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j)
      for (int k = 0; k < 128; ++k) ref[i * 16 + j] += (double)Af[i * 128 + k] * Bf[k * 16 + j];
  uint8_t *dA, *dB; float* dO;
  CK(hipMalloc(&dA, 2048)); CK(hipMalloc(&dB, 2048)); CK(hipMalloc(&dO, 1024));
  CK(hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), 2048, hipMemcpyHostToDevice));
  struct { const char* name; int mode, sa, sb; } runs[] = {
      {"literal 0,0", 0, 0, 0},          {"literal 127,127", 1, 0, 0},     {"runtime 0,0", 2, 0, 0},
      {"runtime 127,127", 2, 127, 127},  {"runtime 128,127", 2, 128, 127}, {"runtime 127,126", 2, 127, 126},
      {"opsel 1/2 bytes", 3, 0x00007f00, 0x00800000}};
  for (auto& r : runs) {
    if (r.mode == 0) probe_scale<0><<<1, 64>>>(dA, dB, r.sa, r.sb, dO);
    if (r.mode == 1) probe_scale<1><<<1, 64>>>(dA, dB, r.sa, r.sb, dO);
    if (r.mode == 2) probe_scale<2><<<1, 64>>>(dA, dB, r.sa, r.sb, dO);
    if (r.mode == 3) probe_scale<3><<<1, 64>>>(dA, dB, r.sa, r.sb, dO);
    CK(hipDeviceSynchronize());
    float o[256];
    CK(hipMemcpy(o, dO, 1024, hipMemcpyDeviceToHost));
    double ratio = 0, maxerr1 = 0;
    int n = 0;
    for (int i = 0; i < 256; ++i)
      if (std::fabs(ref[i]) > 1) { ratio += o[i] / ref[i]; ++n; }
    ratio /= n;
    for (int i = 0; i < 256; ++i) maxerr1 = std::fmax(maxerr1, std::fabs(o[i] - ratio * ref[i]));
    printf("scale %-18s: mean out/ref %.6g, max|out - ratio*ref| %.3g  (o[0]=%g ref[0]=%g)\n", r.name, ratio, maxerr1,
           o[0], ref[0]);
  }
  return 0;
}
