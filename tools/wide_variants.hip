// Variant harness for the matrix-core apply at five K steps (65 <= k <= 80,
// uniform input offsets: the encodes), tools only: the product kernel's walk
// (rs_apply_mfma_kernel.hpp) instantiated at other tile widths, column passes,
// refill styles and waves per SIMD, launched on caller buffers so that
// tools/wide_variants.py times them in interleaved rounds in one process.
//
//   make widevar && python tools/wide_variants.py --need 80 --total 100
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "mfma_table.hpp"
#include "rs_apply_mfma_kernel.hpp"

using namespace slime;
using namespace slime::apply;

namespace {

template <int KS, int W, int NH, int WAVES>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void wv_kernel(
    const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t in_obj_stride, uint64_t in_shard,
    uint64_t out_obj_stride, uint64_t out_shard, const uint8_t* __restrict__ table,
    const uint32_t* __restrict__ out_idx, uint64_t ncols, uint32_t nobj, uint32_t rows, uint32_t k, uint32_t nseg) {
  extern __shared__ i32x4 lds[];
  const uint32_t MT = (rows + 3) / 4;
  const uint32_t lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
  uint64_t* lrowc;
  uint32_t* loff;
  ShardOffs<KS, true> so;
  mfma_prologue(lds, table, nullptr, out_idx, in_shard * 4, out_shard * 4, MT, KS, rows, k, g, &lrowc, &loff, so);
  const uint32_t nvec = (uint32_t)(ncols >> 2);
  const uint32_t seg_vec = segment_vectors(nvec, nseg);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint32_t wave = blockIdx.x * kWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWaves;
  NoPre nopre;
  for (uint64_t wi = blockIdx.y; wi < nwork; wi += gridDim.y) {
    const uint64_t obj = wi / nseg;
    const uint32_t seg = (uint32_t)(wi % nseg);
    const char* __restrict__ ib = reinterpret_cast<const char*>(in + obj * in_obj_stride);
    char* __restrict__ ob = reinterpret_cast<char*>(out + obj * out_obj_stride);
    const uint32_t v0 = seg * seg_vec < nvec ? seg * seg_vec : nvec;
    const uint32_t v1 = nvec - v0 > seg_vec ? v0 + seg_vec : nvec;
    if (v1 > v0)
      mfma_walk<KS, W, true, true, false, NoPre, ShardOffs<KS, true>, NH>(
          ib, ob, so, lds, lrowc, loff, MT, rows, lane, g, n, 4 * v0, 4 * v1, wave, nwaves, MfmaIO{0x80808080u, 0u},
          nopre);
  }
}

template <int KS, int W, int NH, int WAVES>
hipError_t launch(const uint32_t* in, uint32_t* out, uint64_t in_obj, uint64_t in_shard, uint64_t out_obj,
                  uint64_t out_shard, const uint8_t* table, const uint32_t* out_idx, uint64_t ncols, uint32_t nobj,
                  uint32_t rows, uint32_t k, hipStream_t s) {
  const uint32_t lds = mfma_lds_bytes(mfma::mtiles(rows), KS);
  // object_segments (rs_apply.hip): about 256 object segments in flight
  const uint64_t want = (256 + nobj - 1) / nobj, max_s = (ncols >> 2) / 1024 ? (ncols >> 2) / 1024 : 1;
  const uint32_t nseg = (uint32_t)(want < max_s ? want : max_s);
  const uint64_t nwork = (uint64_t)nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  uint64_t gx = (256ull * WAVES + gy - 1) / gy;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((wv_kernel<KS, W, NH, WAVES>), dim3((uint32_t)gx, (uint32_t)gy), dim3(kBlock), lds, s, in,
                     out, in_obj, in_shard, out_obj, out_shard, table, out_idx, ncols, nobj, rows, k, nseg);
  return hipGetLastError();
}

}  // namespace

extern "C" {

// Variant names, one per id (nullptr past the last).
const char* wv_name(int v) {
  // (split refills -- each column pass's half reloaded right after it -- ran 0.36 of peak: removed)
  static const char* names[] = {"W4 NH2 2w", "W2 NH1 2w", "W4 NH1 1w (product)", "W4 NH1 2w (spills)"};
  return v >= 0 && v < (int)(sizeof(names) / sizeof(names[0])) ? names[v] : nullptr;
}

// Host-side digit table of coeff (rows x k) into dst (capacity cap); its size.
uint64_t wv_table(const uint32_t* coeff, uint32_t rows, uint32_t k, uint8_t* dst, uint64_t cap) {
  const std::vector<uint8_t> t = mfma::build_table(coeff, rows, k, false);
  if (dst && cap >= t.size()) memcpy(dst, t.data(), t.size());
  return t.size();
}

int wv_launch(int v, const uint32_t* in, uint32_t* out, uint64_t in_obj, uint64_t in_shard, uint64_t out_obj,
              uint64_t out_shard, const uint8_t* table, const uint32_t* out_idx, uint64_t ncols, uint32_t nobj,
              uint32_t rows, uint32_t k, hipStream_t s) {
  if (mfma::ksteps(k) != 5 || rows > 32 || (ncols & 63)) return (int)hipErrorInvalidValue;
#define WV(W, NH, WV_) \
  launch<5, W, NH, WV_>(in, out, in_obj, in_shard, out_obj, out_shard, table, out_idx, ncols, nobj, rows, k, s)
  switch (v) {
    case 0: return (int)WV(4, 2, 2);
    case 1: return (int)WV(2, 1, 2);
    case 2: return (int)WV(4, 1, 1);
    case 3: return (int)WV(4, 1, 2);
    default: return (int)hipErrorInvalidValue;
  }
#undef WV
}

}  // extern "C"
