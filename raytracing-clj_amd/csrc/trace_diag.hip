// trace_diag.hip — the diagnostic library's kernels (librtclj_diag.so only;
// the product library, trace.hip, carries none of them): the A/B scans of
// the sphere table, the direction-coherent waves (sorted_kernel, variants 20
// and 21: measured slower) and the statistics builds of the
// product traversals (variants 3, 6, 7, 10, 13, 17, 19: the same kernel with
// event and flop counters, which bench.py's roofline reads).  Every variant
// renders the product kernel's bits.
#include "trace_kernel.h"

namespace rtclj {

// The linear scans over the sphere table (the diagnostic variants 1-3, 8-10):
// every body tested, in body order (hittable.clj:7-31 via raytracing.clj:33-43).
template <int SRC, int SCAN, class F>
__device__ void diag_scan(const KArgs& a, const float4* s_geo, float ox, float oy, float oz, float ux, float uy,
                          float uz, F&& consider) {
  const int n = a.n;
  if constexpr (SCAN == SCAN_SIMPLE) {
#pragma unroll 1
    for (int s = 0; s < n; ++s) {
      float4 g;
      if constexpr (SRC == SRC_LDS) g = s_geo[s];
      else g = a.geo[s];
      // hittable.clj:10-14 with a unit direction: a = 1, h = u.oc,
      // c = |oc|^2 - r^2 (y first: the big ground sphere cancels exactly in the fma)
      const float ocx = g.x - ox, ocy = g.y - oy, ocz = g.z - oz;
      const float h = fmaf(uz, ocz, fmaf(uy, ocy, ux * ocx));
      const float c = fmaf(ocx, ocx, fmaf(ocz, ocz, fmaf(ocy, ocy, g.w)));
      const float disc = fmaf(h, h, -c);
      // h < 0 && c >= 0: both roots <= 0 (exact in fp: sqrt(RN(h*h)) = |h|)
      if ((disc >= 0.0f) & ((h >= 0.0f) | (c < 0.0f))) consider(h, disc, s);
    }
  } else {
    // As SCAN_GROUP4, but the arithmetic of two bodies runs in one packed
    // instruction (v_pk_add/mul/fma_f32: each half is the same IEEE-rounded
    // op as the scalar form, so the bits are unchanged); the group's
    // "any candidate" test is one max-reduction and one compare.
    const Pair* tab;
    if constexpr (SRC == SRC_LDS) tab = reinterpret_cast<const Pair*>(s_geo);
    else tab = a.geo2;
    const f2 ox2 = {ox, ox}, oy2 = {oy, oy}, oz2 = {oz, oz};
    const f2 ux2 = {ux, ux}, uy2 = {uy, uy}, uz2 = {uz, uz};
    Pair A = tab[0], B = tab[1];
    for (int s = 0; s < n; s += 4) {
      const Pair nA = tab[(s >> 1) + 2], nB = tab[(s >> 1) + 3];
      f2 h[2], c[2], disc[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const Pair& g = j == 0 ? A : B;
        const f2 ocx = g.x - ox2, ocy = g.y - oy2, ocz = g.z - oz2;
        h[j] = fma2(uz2, ocz, fma2(uy2, ocy, ux2 * ocx));
        c[j] = fma2(ocx, ocx, fma2(ocz, ocz, fma2(ocy, ocy, g.w)));
        disc[j] = fma2(h[j], h[j], -c[j]);
      }
      const float q0 = fminf(disc[0].x, fmaxf(h[0].x, -c[0].x));
      const float q1 = fminf(disc[0].y, fmaxf(h[0].y, -c[0].y));
      const float q2 = fminf(disc[1].x, fmaxf(h[1].x, -c[1].x));
      const float q3 = fminf(disc[1].y, fmaxf(h[1].y, -c[1].y));
      if (fmaxf(fmaxf(q0, q1), fmaxf(q2, q3)) >= 0.0f) {
        if (q0 >= 0.0f) consider(h[0].x, disc[0].x, s);
        if (q1 >= 0.0f) consider(h[0].y, disc[0].y, s + 1);
        if (q2 >= 0.0f) consider(h[1].x, disc[1].x, s + 2);
        if (q3 >= 0.0f) consider(h[1].y, disc[1].y, s + 3);
      }
      A = nA;
      B = nB;
    }
  }
}

// ------------------------------------------------ direction-coherent waves ----
// sorted_kernel<SORT> (variants 20 / 21; DESIGN.md §3.6, an A/B against the
// default traversal 16).  The same sample pool, traversal (the 4-body-leaf
// BVH in LDS), shading and fixed-point sums as trace_kernel, in a different
// execution shape: a 512-thread workgroup (8 waves) owns an 8 x 16-pixel
// tile, and its waves advance in lock step, one ray-color level per
// iteration.  Before every iteration the workgroup's 512 paths are dealt to
// its waves in key order -- fresh camera samples first, then the bounce
// paths by the octant of their direction (SORT; without it only the live
// paths are packed into the first waves) -- through an exchange buffer in
// LDS, so that a wave's lanes traverse the tree in similar directions
// (tools/simt_sim.cpp priced it: 59.3 against 66.5 VALU per sample for the
// shipped shape).  Paths without a path state (the pool's drain) sink to the
// last waves, which skip the iteration: the exchange is also the drain's
// compaction.  One tree copy serves 8 waves, so the exchange buffer fits
// beside it at 3 workgroups (6 waves per SIMD) per CU.
//
// Exchange buffer ([wave][field][lane] u32, 11 fields a path): a fresh
// sample is its pool index (field 0); a bounce path is origin, direction,
// throughput, RNG state and (pixel | depth left << 7 | (body left + 1) << 17).
// After the exchange a wave's traversal stack lives in its own slots of the
// buffer (it has read them before it pushes).
template <bool SORT>
__global__ __launch_bounds__(kSortThreads, 6) void sorted_kernel(const KArgs a) {
  __shared__ int s_pool_next;
  __shared__ unsigned long long s_segs;
  __shared__ unsigned long long s_acc[kSortNPX * 3];
  __shared__ float4 s_px[kSortNPX];
  __shared__ int s_cnt[kSortWaves * kSortKeys];
  extern __shared__ __attribute__((aligned(16))) float4 s_geo[];
  uint64_t st_t0 = 0;
  const int lane = threadIdx.x & 63;
  const int wv = static_cast<int>(threadIdx.x >> 6);
  const int unit = static_cast<int>(blockIdx.x);
  const KArgsP ka = kargs_opaque();
  for (int i = threadIdx.x; i < a.bvh_blob_f4; i += kSortThreads) s_geo[i] = a.bvh_blob[i];
  if (ka->tile_cost) st_t0 = __builtin_amdgcn_s_memrealtime();
  // the unit: a whole tile, or one sample split of a tile (as trace_kernel)
  int pos = unit, split_ix = 0, nsplit = 1, tile;
  const bool split = unit >= ka->n_whole;
  if (split && ka->unit_tab) {
    const int2 u = ka->unit_tab[unit - ka->n_whole];
    if (u.x < 0) return;
    tile = u.x;
    split_ix = u.y & 255;
    nsplit = u.y >> 8;
  } else {
    if (split) {
      const int v = unit - ka->n_whole;
      const int t = v / ka->split;
      pos = ka->n_whole + t;
      split_ix = v - t * ka->split;
      nsplit = ka->split;
    }
    tile = ka->tile_order ? ka->tile_order[pos] : pos;
  }
  const int tby = tile / ka->tiles_x, tbx = tile - tby * ka->tiles_x;
  const int qx0 = tbx * kTile, qy0 = tby * kSortTH;
  const int vw = max(0, min(kTile, ka->width - qx0));
  const int vh = max(0, min(kSortTH, ka->rows_out - qy0));
  const int npx = vw * vh;
  auto image_row = [&](int r) {
    if (a.tile_step > 0) {
      const int t = div_magic(r, a.rt_magic);
      return a.row_begin + (a.tile_first + t * a.tile_step) * a.row_tile + (r - t * a.row_tile);
    }
    return a.row_begin + r;
  };
  auto pixel_key = [&](int x, int y) {
    return mix32(a.key ^ mix32(static_cast<uint32_t>(y) * static_cast<uint32_t>(a.width) + static_cast<uint32_t>(x)));
  };
  const float cx = a.cam[0], cy = a.cam[1], cz = a.cam[2];
  const int k0 = split ? static_cast<int>(static_cast<int64_t>(split_ix) * ka->spp / nsplit) : 0;
  const int cnt = split ? static_cast<int>(static_cast<int64_t>(split_ix + 1) * ka->spp / nsplit) - k0 : ka->spp;
  const int pool = (cnt > 0 && ka->max_depth > 0) ? npx * cnt : 0;
  const uint32_t mag_vw = vw > 0 ? 0xffffffffu / static_cast<uint32_t>(vw) + 1u : 0u;
  const uint64_t npx_magic = npx > 1 ? ~0ull / static_cast<uint64_t>(npx) + 1ull : 0ull;
  if (threadIdx.x == 0) {
    s_pool_next = 0;
    s_segs = 0ull;
  }
  if (threadIdx.x < kSortNPX * 3) s_acc[threadIdx.x] = 0ull;
  {
    const int t = static_cast<int>(threadIdx.x);
    if (t < npx) {
      const int qy = vw == 1 ? t : static_cast<int>(__umulhi(static_cast<uint32_t>(t), mag_vw));
      const int px = qx0 + (t - qy * vw);
      const int gy = image_row(qy0 + qy);
      s_px[t] = make_float4(__uint_as_float(pixel_key(px, gy)), static_cast<float>(px), static_cast<float>(gy), 0.0f);
    }
  }
  __syncthreads();

  uint32_t* const xw = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s_geo) + a.bvh_blob_f4 * 16);
  auto xslot = [&](int slot, int f) -> uint32_t* { return xw + ((slot >> 6) * kXFields + f) * 64 + (slot & 63); };
  // j: >= 0 a fresh sample (pool index), -1 a path in progress, -2 none
  int j = -2, q = 0;
  uint32_t st = 0;
  float ox = 0, oy = 0, oz = 0, dx = 0, dy = 0, dz = 0;
  float tr = 1, tg = 1, tb = 1;
  int rem = 0, last = -1;
  bool spent = pool == 0;   // wave-uniform: the pool is handed out
  uint32_t segs = 0;
  const KNode* nodes = reinterpret_cast<const KNode*>(s_geo);
  const Pair* pairs = reinterpret_cast<const Pair*>(reinterpret_cast<const char*>(s_geo) + a.bvh_off_pairs);
  const int2* pidx = reinterpret_cast<const int2*>(reinterpret_cast<const char*>(s_geo) + a.bvh_off_pidx);
  // this wave's traversal stack: its own exchange slots, [entry][lane] u16
  unsigned short* const stk0 = reinterpret_cast<unsigned short*>(xw + wv * kXWaveWords) + lane;

  for (;;) {
    // ---- refill: lanes without a path take the next pool indices ----
    if (!spent) {
      const uint64_t m = __ballot(j == -2);
      if (m) {
        const int need = static_cast<int>(__popcll(m));
        const int rank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
        int g = 0;
        if (lane == 0) g = atomicAdd(&s_pool_next, need);
        g = __builtin_amdgcn_readlane(g, 0);
        if (j == -2) j = g + rank < pool ? g + rank : -2;
        spent = g + need >= pool;
      }
    }
    // ---- deal the workgroup's paths to its waves in key order ----
    int key = 9;
    if (j >= 0) key = 0;
    else if (j == -1) key = SORT ? 1 + ((dx < 0.0f) ? 1 : 0) + ((dy < 0.0f) ? 2 : 0) + ((dz < 0.0f) ? 4 : 0) : 1;
    uint64_t mine = 0;
    int mycnt = 0;
#pragma unroll
    for (int k = 0; k < kSortKeys; ++k) {
      if (!SORT && k >= 2 && k < 9) continue;
      const uint64_t b = __ballot(key == k);
      mine = key == k ? b : mine;
      mycnt = lane == k ? static_cast<int>(__popcll(b)) : mycnt;
    }
    const int myrank = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(mine >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(mine), 0u)));
    if (lane < kSortKeys) s_cnt[wv * kSortKeys + lane] = mycnt;
    __syncthreads();
    // lane k < 10: key k's count over the waves, and in the waves before this one
    int tot = 0, before = 0;
    if (lane < kSortKeys) {
#pragma unroll
      for (int w2 = 0; w2 < kSortWaves; ++w2) {
        const int c = s_cnt[w2 * kSortKeys + lane];
        tot += c;
        before += w2 < wv ? c : 0;
      }
    }
    int scan = tot;   // inclusive prefix over the keys (lanes 0..9)
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const int v = __shfl_up(scan, off);
      scan += lane >= off ? v : 0;
    }
    const int n_live = __builtin_amdgcn_readlane(scan, 8);    // keys 0..8: the paths and fresh samples
    const int n_fresh = __builtin_amdgcn_readlane(tot, 0);
    if (n_live == 0) break;   // (workgroup-uniform: every wave read the same counts)
    const int base_k = scan - tot + before;                   // lane k: this wave's first slot of key k
    const int dst = __shfl(base_k, key) + myrank;
    if (key == 0) {
      *xslot(dst, 0) = static_cast<uint32_t>(j);
    } else if (key < 9) {
      *xslot(dst, 0) = __float_as_uint(ox);
      *xslot(dst, 1) = __float_as_uint(oy);
      *xslot(dst, 2) = __float_as_uint(oz);
      *xslot(dst, 3) = __float_as_uint(dx);
      *xslot(dst, 4) = __float_as_uint(dy);
      *xslot(dst, 5) = __float_as_uint(dz);
      *xslot(dst, 6) = __float_as_uint(tr);
      *xslot(dst, 7) = __float_as_uint(tg);
      *xslot(dst, 8) = __float_as_uint(tb);
      *xslot(dst, 9) = st;
      *xslot(dst, 10) = static_cast<uint32_t>(q) | (static_cast<uint32_t>(rem) << 7) |
                        (static_cast<uint32_t>(last + 1) << 17);
    }
    __syncthreads();
    {
      const int t = static_cast<int>(threadIdx.x);
      if (t < n_fresh) {
        j = static_cast<int>(*xslot(t, 0));
      } else if (t < n_live) {
        ox = __uint_as_float(*xslot(t, 0));
        oy = __uint_as_float(*xslot(t, 1));
        oz = __uint_as_float(*xslot(t, 2));
        dx = __uint_as_float(*xslot(t, 3));
        dy = __uint_as_float(*xslot(t, 4));
        dz = __uint_as_float(*xslot(t, 5));
        tr = __uint_as_float(*xslot(t, 6));
        tg = __uint_as_float(*xslot(t, 7));
        tb = __uint_as_float(*xslot(t, 8));
        st = *xslot(t, 9);
        const uint32_t meta = *xslot(t, 10);
        q = static_cast<int>(meta & 127u);
        rem = static_cast<int>((meta >> 7) & 1023u);
        last = static_cast<int>(meta >> 17) - 1;
        j = -1;
      } else {
        j = -2;
      }
    }
    if (wv * 64 >= n_live) continue;   // (wave-uniform: no path in this wave; the barriers above)
    if (j < -1) continue;
    // ---- a fresh sample: compute-pixel's camera ray (raytracing.clj:144-151) ----
    if (j >= 0) {
      const int k = div_magic(j, npx_magic);
      q = j - k * npx;
      const float4 pt = s_px[q];
      st = mix32(__float_as_uint(pt.x) + static_cast<uint32_t>(a.sample_begin + k0 + k) * 0x9e3779b9u);
      if (st == 0) st = 0x6d2b79f5u;
      const float fx = pt.y + rng_centered(st);
      const float fy = pt.z + rng_centered(st);
      const float sx = fmaf(a.cam[9], fy, fmaf(a.cam[6], fx, a.cam[3]));
      const float sy = fmaf(a.cam[10], fy, fmaf(a.cam[7], fx, a.cam[4]));
      const float sz = fmaf(a.cam[11], fy, fmaf(a.cam[8], fx, a.cam[5]));
      if (a.defocus) {
        float qx, qy2;
        if (a.sampler & RT_SAMPLER_DISK) {
          disk_direct(st, qx, qy2);
        } else {
          do {
            qx = rng_sym(st);
            qy2 = rng_sym(st);
          } while (!(fmaf(qy2, qy2, qx * qx) < 1.0f));
        }
        ox = fmaf(a.cam[15], qy2, fmaf(a.cam[12], qx, cx));
        oy = fmaf(a.cam[16], qy2, fmaf(a.cam[13], qx, cy));
        oz = fmaf(a.cam[17], qy2, fmaf(a.cam[14], qx, cz));
      } else {
        ox = cx;
        oy = cy;
        oz = cz;
      }
      dx = sx - ox;
      dy = sy - oy;
      dz = sz - oz;
      tr = tg = tb = 1.0f;
      rem = a.max_depth;
      last = -1;
      j = -1;
    }
    // ---- one ray-color level (as trace_kernel's SCAN_BVHQ iteration) ----
    bool done = false;
    --rem;
    ++segs;
    const float len = sqrt_rn(fmaf(dz, dz, fmaf(dy, dy, dx * dx)));
    const float il = 1.0f / len;
    const float ux = dx * il, uy = dy * il, uz = dz * il;
    const float tmin = 1e-3f * len;
    float best_t = INFINITY;
    int best = -1;
    {
      auto consider_tie = [&](float h, float disc, int s) {
        const float sq = (s == last) ? fabsf(h) : sqrt_rn(disc);
        const float tn = h - sq;
        const float t = tn > tmin ? tn : h + sq;
        const uint64_t kk = (static_cast<uint64_t>(__float_as_uint(t)) << 32) | static_cast<uint32_t>(s);
        const uint64_t bkey = (static_cast<uint64_t>(__float_as_uint(best_t)) << 32) | static_cast<uint32_t>(best);
        const bool acc = (t > tmin) & (kk < bkey);
        best_t = acc ? t : best_t;
        best = acc ? s : best;
      };
      const float ecx = ox - a.bvh_c[0], ecy = oy - a.bvh_c[1], ecz = oz - a.bvh_c[2];
      const float D = __builtin_amdgcn_sqrtf(fmaf(ecz, ecz, fmaf(ecy, ecy, ecx * ecx))) + a.bvh_r;
      const float P = fmaf(2e-3f, D, 1e-6f);
      const float rux = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(ux), -1e24f, 1e24f);
      const float ruy = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(uy), -1e24f, 1e24f);
      const float ruz = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(uz), -1e24f, 1e24f);
      f2 r_xy = {rux, ruy}, r_z = {ruz, ruz};
      const float nlx = -(ecx + P) * rux, nly = -(ecy + P) * ruy, nlz = -(ecz + P) * ruz;
      const float nhx = -(ecx - P) * rux, nhy = -(ecy - P) * ruy, nhz = -(ecz - P) * ruz;
      const bool sx = rux < 0.0f, sy = ruy < 0.0f, sz = ruz < 0.0f;
      f2 nf_x = {sx ? nhx : nlx, sx ? nlx : nhx};
      f2 nf_y = {sy ? nhy : nly, sy ? nly : nhy};
      f2 nf_z = {sz ? nhz : nlz, sz ? nlz : nhz};
      const int offx = sx ? 8 : 0, offy = 24 + (sy ? 8 : 0), offz = 48 + (sz ? 8 : 0);
      f2 o_xy = {ox, oy}, o_zux = {oz, ux}, u_yz = {uy, uz};
      auto leaf = [&](int p) {
        float hh[4], dd[4];
        int ii[4];
        unsigned nc[4];
        const Pair* const lp = pairs + p;
        const int2* const li = pidx + p;
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
          const Pair g = lp[qq];
          const int2 id = li[qq];
          asm volatile("" : "+v"(o_xy), "+v"(o_zux), "+v"(u_yz));
          const f2 ocx = g.x - bc_lo(o_xy), ocy = g.y - bc_hi(o_xy), ocz = g.z - bc_lo(o_zux);
          const f2 h = fma2(bc_hi(u_yz), ocz, fma2(bc_lo(u_yz), ocy, bc_hi(o_zux) * ocx));
          const f2 c = fma2(ocx, ocx, fma2(ocz, ocz, fma2(ocy, ocy, g.w)));
          const f2 disc = fma2(h, h, -c);
          hh[2 * qq] = h.x;
          hh[2 * qq + 1] = h.y;
          dd[2 * qq] = disc.x;
          dd[2 * qq + 1] = disc.y;
          ii[2 * qq] = id.x;
          ii[2 * qq + 1] = id.y;
          const float d0 = disc.x, d1 = disc.y, h0 = h.x, h1 = h.y, c0 = c.x, c1 = c.y;
          nc[2 * qq] = __builtin_amdgcn_bitop3_b32(__float_as_uint(d0), __float_as_uint(h0), __float_as_uint(c0), 0x0b);
          nc[2 * qq + 1] = __builtin_amdgcn_bitop3_b32(__float_as_uint(d1), __float_as_uint(h1), __float_as_uint(c1), 0x0b);
        }
        const unsigned b01 = __builtin_amdgcn_perm(nc[1], nc[0], 0x0c0c0b09u);
        const unsigned b23 = __builtin_amdgcn_perm(nc[3], nc[2], 0x0b090c0cu);
        unsigned m = __builtin_amdgcn_bitop3_b32(b01, b23, 0x01010101u, 0xa8);
        while (m) {
          const unsigned k = __builtin_ctz(m);
          m &= m - 1;
          float h = hh[0], d = dd[0];
          int s = ii[0];
#pragma unroll
          for (int jj = 1; jj < 4; ++jj) {
            h = k == static_cast<unsigned>(8 * jj) ? hh[jj] : h;
            d = k == static_cast<unsigned>(8 * jj) ? dd[jj] : d;
            s = k == static_cast<unsigned>(8 * jj) ? ii[jj] : s;
          }
          consider_tie(h, d, s);
        }
      };
      auto node_test = [&](int node, float& tn0, float& tn1, bool& hit0, bool& hit1, int& c0, int& c1) {
        const char* nb = reinterpret_cast<const char*>(nodes) + static_cast<unsigned>(node);
        const f2* ax = reinterpret_cast<const f2*>(nb + offx);
        const f2* ay = reinterpret_cast<const f2*>(nb + offy);
        const f2* az = reinterpret_cast<const f2*>(nb + offz);
        const int2 ch = *reinterpret_cast<const int2*>(nb + 72);
        asm volatile("" : "+v"(r_xy), "+v"(r_z), "+v"(nf_x), "+v"(nf_y), "+v"(nf_z));
        const f2 tnx = fma2(ax[0], bc_lo(r_xy), bc_lo(nf_x)), tfx = fma2(ax[1], bc_lo(r_xy), bc_hi(nf_x));
        const f2 tny = fma2(ay[0], bc_hi(r_xy), bc_lo(nf_y)), tfy = fma2(ay[1], bc_hi(r_xy), bc_hi(nf_y));
        const f2 tnz = fma2(az[0], bc_lo(r_z), bc_lo(nf_z)), tfz = fma2(az[1], bc_lo(r_z), bc_hi(nf_z));
        tn0 = fmaxf(fmaxf(tnx.x, tny.x), tnz.x);
        tn1 = fmaxf(fmaxf(tnx.y, tny.y), tnz.y);
        const float tf0 = fminf(fminf(tfx.x, tfy.x), tfz.x);
        const float tf1 = fminf(fminf(tfx.y, tfy.y), tfz.y);
        float ntn0, ntn1;
        asm("v_max_f32 %0, %1, %2" : "=v"(ntn0) : "v"(tn0), "v"(tmin));
        asm("v_max_f32 %0, %1, %2" : "=v"(ntn1) : "v"(tn1), "v"(tmin));
        hit0 = ntn0 <= fminf(tf0, best_t);
        hit1 = ntn1 <= fminf(tf1, best_t);
        c0 = ch.x;
        c1 = ch.y;
      };
      for (int b = 0; b < a.n_big_leaves; ++b) leaf(a.big_pair0 + b * 2);
      int node = 0;
      unsigned short* top = stk0;
      bool go = true;
      while (go) {
        float tn0, tn1;
        bool hit0, hit1;
        int c0, c1;
        node_test(node, tn0, tn1, hit0, hit1, c0, c1);
        const bool l0 = hit0 && c0 < 0, l1 = hit1 && c1 < 0;
        if (l0 || l1) {
          leaf(l0 ? ~c0 : ~c1);
          if (l0 && l1) leaf(~c1);
        }
        const bool i0 = hit0 && !l0, i1 = hit1 && !l1;
        const bool sw = tn1 < tn0;
        int nxt = (i0 && (!i1 || !sw)) ? c0 : c1;
        *top = static_cast<unsigned short>(sw ? c0 : c1);
        top += (i0 && i1) ? 64 : 0;
        if (!(i0 || i1)) {
          go = top != stk0;
          top -= go ? 64 : 0;
          nxt = *top;
        }
        node = nxt;
      }
    }
    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    if (best < 0) {
      const float sa = 0.5f * (uy + 1.0f);
      const float om = 1.0f - sa;
      cr = tr * fmaf(sa, 0.5f, om);
      cg = tg * fmaf(sa, 0.7f, om);
      cb = tb * fmaf(sa, 1.0f, om);
      done = true;
    } else if (rem == 0) {
      done = true;
    } else {
      const float4 sp = a.sph[best];
      const float hx = fmaf(ux, best_t, ox);
      const float hy = fmaf(uy, best_t, oy);
      const float hz = fmaf(uz, best_t, oz);
      float nx = (hx - sp.x) * sp.w, ny = (hy - sp.y) * sp.w, nz = (hz - sp.z) * sp.w;
      const bool front = fmaf(dz, nz, fmaf(dy, ny, dx * nx)) < 0.0f;
      if (!front) {
        nx = -nx;
        ny = -ny;
        nz = -nz;
      }
      const int kind = a.kind[best];
      const float4 m = a.mat[best];
      ox = hx;
      oy = hy;
      oz = hz;
      last = best;
      if (kind == RT_LAMBERTIAN || kind == RT_METAL) {
        float qx, qy, qz;
        if (a.sampler & RT_SAMPLER_SPHERE)
          sphere_direct(st, qx, qy, qz);
        else
          random_unit<false>(st, qx, qy, qz);
        if (kind == RT_LAMBERTIAN) {
          float sx = qx + nx, sy = qy + ny, sz = qz + nz;
          if (!a.realm && fabsf(sx) < 1e-8f && fabsf(sy) < 1e-8f && fabsf(sz) < 1e-8f) {
            sx = nx;
            sy = ny;
            sz = nz;
          }
          dx = sx;
          dy = sy;
          dz = sz;
          tr *= m.x;
          tg *= m.y;
          tb *= m.z;
        } else {
          const float k2 = 2.0f * fmaf(dz, nz, fmaf(dy, ny, dx * nx));
          const float rx0 = fmaf(-nx, k2, dx), ry0 = fmaf(-ny, k2, dy), rz0 = fmaf(-nz, k2, dz);
          const float rx = fmaf(m.w, qx, rx0), ry = fmaf(m.w, qy, ry0), rz = fmaf(m.w, qz, rz0);
          if (fmaf(rz, nz, fmaf(ry, ny, rx * nx)) > 0.0f) {
            dx = rx;
            dy = ry;
            dz = rz;
            tr *= m.x;
            tg *= m.y;
            tb *= m.z;
          } else {
            done = true;
          }
        }
      } else if (kind == RT_NONE) {
        done = true;
      } else {
        const float ri = front ? m.x : m.w;
        const float r0 = front ? m.y : m.z;
        const float un = fmaf(uz, nz, fmaf(uy, ny, ux * nx));
        const float cosv = fminf(-un, 1.0f);
        const float sinv = sqrt_rn(fmaf(-cosv, cosv, 1.0f));
        bool refl = !(ri * sinv <= 1.0f);
        if (!refl && !a.realm) {
          const float xi = rng_uniform(st);
          const float x1 = 1.0f - cosv;
          const float x2 = x1 * x1;
          const float x5 = x2 * x2 * x1;
          refl = fmaf(1.0f - r0, x5, r0) > xi;
        }
        if (refl) {
          const float k2 = 2.0f * un;
          dx = fmaf(-nx, k2, ux);
          dy = fmaf(-ny, k2, uy);
          dz = fmaf(-nz, k2, uz);
        } else {
          const float qx = fmaf(nx, cosv, ux) * ri;
          const float qy = fmaf(ny, cosv, uy) * ri;
          const float qz = fmaf(nz, cosv, uz) * ri;
          const float par = -sqrt_rn(fabsf(1.0f - fmaf(qz, qz, fmaf(qy, qy, qx * qx))));
          dx = fmaf(nx, par, qx);
          dy = fmaf(ny, par, qy);
          dz = fmaf(nz, par, qz);
        }
      }
    }
    if (done) {
      unsigned long long* acc = &s_acc[q * 3];
      __hip_atomic_fetch_add(acc + 0, static_cast<unsigned long long>(fix24(cr)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(acc + 1, static_cast<unsigned long long>(fix24(cg)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(acc + 2, static_cast<unsigned long long>(fix24(cb)), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      j = -2;
    }
  }

  // ---- per-pixel mean (compute-pixel's accum / spp, raytracing.clj:155) ----
  __syncthreads();
  const KArgsP ke = kargs_opaque();
  const int t = static_cast<int>(threadIdx.x);
  if (t < npx * 3) {
    const int fp = t / 3, ch = t - 3 * fp;
    const int qy = vw == 1 ? fp : static_cast<int>(__umulhi(static_cast<uint32_t>(fp), mag_vw));
    const int px = qx0 + (fp - qy * vw), ro = qy0 + qy;
    const size_t e = (static_cast<size_t>(ro) * ke->width + px) * 3 + ch;
    if (split) {
      if (s_acc[t]) __hip_atomic_fetch_add(&ke->part[e], s_acc[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const float tot = static_cast<float>(s_acc[t]) * 0x1p-24f;
      const float inv = static_cast<float>(ke->spp > 0 ? ke->spp : 1);
      ke->out[e] = ke->realm ? tot * (1.0f / inv) : tot / inv;
    }
  }
  if (ke->tile_cost && threadIdx.x == 0) {
    const uint64_t dt = __builtin_amdgcn_s_memrealtime() - st_t0;
    atomicAdd(&ke->tile_cost[tile], static_cast<unsigned>(dt < 0xffffffffull ? dt : 0xffffffffull));
  }
  if (ke->counters && threadIdx.x == 0 && pool) atomicAdd(&ke->counters[1], static_cast<unsigned long long>(pool));
  if (a.counters) {
    uint32_t v = segs;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0 && v) atomicAdd(&s_segs, static_cast<unsigned long long>(v));
    __syncthreads();
    if (threadIdx.x == 0 && s_segs) atomicAdd(&a.counters[0], s_segs);
  }
}


// the diagnostic variants (trace.hip's variant_table asks here for all but
// 0, 5, 12, 16, 18 and 22)
const Variant* diag_variant(int v) {
  static const Variant t[] = {
      {nullptr, false, false, 0},                                          // 0 (product)
      {RT_K(SRC_LDS, SCAN_SIMPLE, false), true, false, SCAN_SIMPLE},       // 1
      {RT_K(SRC_SCALAR, SCAN_SIMPLE, false), false, false, SCAN_SIMPLE},   // 2
      {RT_K(SRC_LDS, SCAN_SIMPLE, true), true, true, SCAN_SIMPLE},         // 3
      {RT_K(SRC_LDS, SCAN_GROUP4, false), true, false, SCAN_GROUP4},       // 4
      {nullptr, false, false, 0},                                          // 5 (product)
      {RT_K(SRC_LDS, SCAN_GROUP4, true), true, true, SCAN_GROUP4},         // 6
      {RT_K(SRC_SCALAR, SCAN_GROUP4, true), false, true, SCAN_GROUP4},     // 7
      {RT_K(SRC_LDS, SCAN_PK4, false), true, false, SCAN_PK4},             // 8
      {RT_K(SRC_SCALAR, SCAN_PK4, false), false, false, SCAN_PK4},         // 9
      {RT_K(SRC_SCALAR, SCAN_PK4, true), false, true, SCAN_PK4},           // 10
      {RT_K(SRC_LDS, SCAN_BVH, false), true, false, SCAN_BVH},             // 11
      {nullptr, false, false, 0},                                          // 12 (product)
      {RT_K(SRC_LDS, SCAN_BVH, true), true, true, SCAN_BVH},               // 13
      {nullptr, false, false, 0},                                          // 14 (dropped: while-while traversal)
      {nullptr, false, false, 0},                                          // 15 (dropped: its stats build)
      {nullptr, false, false, 0},                                          // 16 (product)
      {RT_K(SRC_LDS, SCAN_BVHQ, true), true, true, SCAN_BVHQ},             // 17
      {nullptr, false, false, 0},                                          // 18 (product)
      {RT_KW(SRC_LDS, SCAN_BVHO, true, 8), true, true, SCAN_BVHO, 512},    // 19
      // direction-coherent waves (A/B, measured slower: profiles/r04/sorted_waves/):
      // octant-sorted, and lock-step packing only
      {reinterpret_cast<const void*>(&sorted_kernel<true>), true, false, SCAN_BVHS, kSortThreads},    // 20
      {reinterpret_cast<const void*>(&sorted_kernel<false>), true, false, SCAN_BVHS, kSortThreads},   // 21
  };
  constexpr int nt = static_cast<int>(sizeof t / sizeof t[0]);
  return (v > 0 && v < nt && t[v].fn) ? &t[v] : nullptr;
}

}  // namespace rtclj
