// Launcher of the matrix-core apply kernel (rs_apply_mfma_kernel.hpp) for wide
// codes: applyMatrix (internal/rs/vector.go:90-102) as an exact int8-limb
// product on v_mfma_i32_16x16x64_i8, for plans whose table carries the digit
// fragments (built for k >= 17 with rows <= 32, k <= 112: mfma_table.hpp).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>

#include "kernels.hpp"
#include "rs_apply_mfma_kernel.hpp"

namespace slime {

// Process-wide switch (slime_rs_kernel_matrix_cores()); on by default.
// Which shapes take the matrix cores is mfma_wanted() below.
static std::atomic<int> g_mfma{1};
int matrix_core_mode() { return g_mfma.load(std::memory_order_relaxed); }
void set_matrix_core_mode(int m) { g_mfma.store(m, std::memory_order_relaxed); }

// Which launches take the matrix cores (product rule, measured on one box,
// profiles/r03/s37_mfma_k32/): every k >= 33, and 17 <= k <= 32 when the
// column's k x rows multiply-accumulates reach 128 -- 24/32 0.646 -> 0.739,
// 32/40 0.676 -> 0.738, while 20/24 (80 per column) ties and 17/20 (51)
// loses 4% (0.739 -> 0.709).
bool mfma_wanted(uint32_t k, uint32_t rows) { return k >= 33 || (k >= 17 && k * rows >= 128); }

bool mfma_eligible(const ApplyLaunch& a) {
  if (!a.mfma || !a.vec_ok || !matrix_core_mode() || !mfma_wanted(a.k, a.rows)) return false;
  if (!mfma::supported(a.rows, a.k)) return false;
  // 32-bit per-lane byte offsets from each object's base (see the kernel).
  const uint64_t lim = 1ull << 32;
  if (((uint64_t)a.in_max * a.in_shard_stride + a.ncols) * 4 >= lim) return false;
  if (((uint64_t)a.out_max * a.out_shard_stride + a.ncols) * 4 >= lim) return false;
  return true;
}

namespace {

// Static tile walk only: a dynamic-schedule form (TicketWalk units of 4 KiB
// per shard, the refill streaming across objects) measured 0-6% slower than
// this walk at 40/48, 48/64, 64/80 and 80/100 (profiles/r03/s33_mfma_queue_bytes/).
// Non-temporal loads and stores (read-once / write-once streams).
template <int KS, bool UNI>
hipError_t launch_ks(const ApplyLaunch& a, hipStream_t stream) {
  const uint32_t mt = mfma::mtiles(a.rows);
  const uint32_t lds = apply::mfma_lds_bytes(mt, KS);
  const uint64_t per_block = 4ull * 16 * 4;  // 4 waves x 16 vectors
  const uint64_t target = 256ull * apply::mfma_waves(KS, apply::mfma_width(KS));  // resident blocks
  // Short objects take one walk over every object's tiles across the whole
  // grid: the per-object walk gives each object a block, most of whose waves
  // have no tile.  4096 objects of 64 columns: 2-3.4x; of 512 columns at five
  // K steps (one wave per SIMD) +25% encode, +7% repair, but at four K steps
  // the per-object walk stays 4% ahead from 8 tiles (profiles/r05/s34_flat/).
  const uint64_t kFlatTiles = apply::mfma_waves(KS, apply::mfma_width(KS)) == 1 ? 32 : 4;
  const uint64_t tc = 16ull * apply::mfma_width(KS);
  const uint64_t tpo = ((a.ncols >> 2) * 4 + tc - 1) / tc;
  if (a.nobj > 1 && tpo <= kFlatTiles) {
    const uint64_t tiles = tpo * a.nobj, nb = (tiles + apply::kWaves - 1) / apply::kWaves;
    const uint64_t gx = std::max<uint64_t>(1, std::min(target, nb));
    hipLaunchKernelGGL((apply::rs_apply_mfma_kernel<KS, true, true, UNI>), dim3((uint32_t)gx), dim3(apply::kBlock),
                       lds, stream, a.in, a.out, a.in_obj_stride, a.in_shard_stride, a.out_obj_stride,
                       a.out_shard_stride, a.mfma, a.coeff, a.in_idx, a.out_idx, a.ncols, a.nobj, a.rows, a.k, 1u, 1u);
    return hipGetLastError();
  }
  const uint32_t nseg = object_segments(a.nobj, a.ncols);
  const uint64_t nwork = (uint64_t)a.nobj * nseg;
  const uint64_t gy = nwork < 65535 ? nwork : 65535;
  uint64_t gx = (target + gy - 1) / gy;
  const uint64_t need = ((a.ncols >> 2) / nseg + per_block - 1) / per_block;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL((apply::rs_apply_mfma_kernel<KS, true, true, UNI>), dim3((uint32_t)gx, (uint32_t)gy),
                     dim3(apply::kBlock), lds, stream, a.in, a.out, a.in_obj_stride, a.in_shard_stride,
                     a.out_obj_stride, a.out_shard_stride, a.mfma, a.coeff, a.in_idx, a.out_idx, a.ncols, a.nobj,
                     a.rows, a.k, nseg, 0u);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_apply_mfma(const ApplyLaunch& a, hipStream_t stream) {
  switch (mfma::ksteps(a.k)) {
    case 1: return launch_ks<1, false>(a, stream);
    case 2: return launch_ks<2, false>(a, stream);
    case 3: return launch_ks<3, false>(a, stream);
    case 4: return launch_ks<4, false>(a, stream);
    // encodes at 65 <= k <= 80 on the uniform offsets
    case 5: return a.in_seq ? launch_ks<5, true>(a, stream) : launch_ks<5, false>(a, stream);
    case 6: return launch_ks<6, false>(a, stream);
    case 7: return launch_ks<7, false>(a, stream);
    default: return hipErrorInvalidValue;  // mfma_eligible() rules this out
  }
}

}  // namespace slime
