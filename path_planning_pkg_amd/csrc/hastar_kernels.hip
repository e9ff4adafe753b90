// hastar_kernels.hip — HIP kernels of the MI355X Hybrid A* planner (gfx950).
//
//   hastar_search_kernel   one wavefront (64 lanes) per planner: the reference's
//                          sequential best-first loop (HybridAStar.cpp:93-199) with its
//                          data-parallel inner work spread over the lanes:
//                          successor APF fields (lanes over obstacles), the 4 Dubins
//                          words of every successor, the holonomic A* neighbour probes,
//                          Dubins-shot sampling + collision check, path reconstruction.
//                          Throughput = many planners per launch (thousands of waves).
//   map kernels            the HBM-bound O(N^2) upkeep of Grid2D/Grid3D: decay,
//                          relocation (rotate + scatter), box/line rasterisation,
//                          node-map (heuristic) initialisation.
//   test kernels           unit-level hooks used by the parity tests.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <type_traits>
#include "hastar_device.h"
#include "hastar_kernels.h"

namespace hastar {

#ifndef HASTAR_WAVES_PER_EU
#define HASTAR_WAVES_PER_EU 2  // search waves per SIMD the register budget must allow
#endif
constexpr int MAXS = 16;   // max steering actions (checked at create)
static_assert(64 / 4 >= MAXS, "4 lanes per candidate action must cover MAXS actions");

// block-placement hints: the inner A*'s rare paths (end of search, duplicates, shape-dependent
// walks, overflows) out of the straight-line common path
#define HASTAR_LIKELY(x) __builtin_expect(!!(x), 1)
#define HASTAR_UNLIKELY(x) __builtin_expect(!!(x), 0)
// Diagnostic build only (-DHASTAR_STAMPS): cycles per phase of the search loop,
// 0 pop+closed insert, 1 successors+APF+Dubins, 2 open/closed bookkeeping, 3 holonomic A*,
// 4 Dubins shot, 5 reconstruct+stats, 6 whole loop, 7 A* in HBM mode, 8-12 LDS A* pop /
// find / insert / unlink-hit / memoise, 13-15 outer find / insert / unlink, 16-18 successor
// generation / APF / Dubins lengths, 19-20 outer insert walk / link, 24 LDS A* pop unlink,
// 25 LDS A* insert link, 30 LDS A* ring insert, 31 LDS A* expansion stores.
#ifdef HASTAR_STAMPS
#define STAMP_T unsigned long long
#define STAMP_NOW() __builtin_amdgcn_s_memtime()
#define STAMP_ADD(slot, t0) (c.cyc[slot] += __builtin_amdgcn_s_memtime() - (t0))
#else
#define STAMP_T int
#define STAMP_NOW() 0
#define STAMP_ADD(slot, t0) ((void)(t0))
#endif

struct Succ {
  float x, y, h, g, vmin;
  int ci, bin, cx, cy;
  float dub;
};

// Pin a wave-uniform value in SGPRs.  The descriptors are read-only kernel arguments, so the
// compiler may re-issue a field's scalar load wherever it runs short of SGPRs
// (rematerialisation) instead of keeping it; each such s_load is followed by an lgkmcnt(0)
// wait, which also drains the wave's outstanding LDS reads.  A value that went through an
// empty asm is opaque: it is kept in a register or spilled to a VGPR lane, never re-loaded.
template <class T>
__device__ __forceinline__ GAS T* pin(GAS T* p) {
  uint64_t v = (uint64_t)p;
  asm volatile("" : "+s"(v));
  return (GAS T*)v;
}
__device__ __forceinline__ uint32_t pin(uint32_t v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ int pin(int v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ float pin(float v) {
  asm volatile("" : "+s"(v));
  return v;
}

struct SearchCtx {
  const PlannerDev* __restrict__ P;   // planner descriptor in HBM (uniform, read-only: scalar loads)
  const SlotArena* __restrict__ A;    // this wave's search arena
  int lane;
  int slot;                  // index of this wave's arena in the device's pool (parks, timing)
  // the hot descriptor fields, pinned in registers for the whole search (bind_hot)
  GAS float* occ;
  GAS float* nm_f;
  GAS uint32_t* visited;
  GAS Cell2* cell2;
  GAS int* prevl;
  GAS Slot3* slots3;
  GAS Closed3* closed3;
  GAS Node3* open3;
  uint32_t smask;
  int N;
  float thr;
  RBT<CachedAcc3> o3;        // outer open tree: HBM nodes behind a register node cache
  PoolState ps3, ps2;
  int n_closed3;
  uint32_t gen3, gen2;
  // 32-bit search statistics (two SGPRs fewer each than 64-bit ones: a search would need
  // hours to count 2^32 pops), widened when they are stored (SearchResult)
  uint32_t pops, succ, apops, asearch, shots, amigr, apops_g;
  int status;
  bool cost_only;   // AStar::a_star_search(get_cost_only): memo exits + memoise (always, inside the search)
  uint32_t prep_epoch;  // latency kernel: the search's epoch in the helper waves' prep table
#ifdef HASTAR_STAMPS
  unsigned long long cyc[NSTAMP];
#endif
};

// Pin a wave-uniform pointer in a VGPR pair instead: the search's SGPRs are its scarce
// registers (the batch kernel spills hundreds of them to VGPR lanes, and the inner A* loop
// reloads them), while its VGPR budget has room.  The map and arena bases below are only ever
// used to form per-lane or uniform global addresses, which a VGPR base serves as well.
template <class T>
__device__ __forceinline__ GAS T* pinv(GAS T* p) {
  uint64_t v = (uint64_t)p;
  asm volatile("" : "+v"(v));
  return (GAS T*)v;
}

// the hot fields of c.P and c.A, once per search (or per A* query).  kVgprMaps: the map and
// cell-record bases in VGPRs (the batch kernel: SGPR spills 740 -> 563 with 32-bit counters,
// +3-5 % expansions/s, profiles/r05d_ab_vgpr_pins.jsonl; the latency kernel keeps them in SGPRs:
// there the VGPR pins cost 9 % on cfg5, profiles/r05f_cfg5_ab.jsonl)
template <bool kVgprMaps = false>
__device__ __forceinline__ void bind_hot(SearchCtx& c) {
  const PlannerDev& P = *c.P;
  const SlotArena& A = *c.A;
  if constexpr (kVgprMaps) {  // (the outer tree's slots3/closed3 stay in SGPRs: in VGPRs they spilled to scratch)
    c.occ = pinv(gp(P.occ));
    c.nm_f = pinv(gp(P.nm_f));
    c.visited = pinv(gp(P.visited));
    c.cell2 = pinv(gp(A.cell2));
    c.prevl = pinv(gp(A.prevl));
    c.slots3 = pin(gp(A.slots3));
    c.closed3 = pin(gp(A.closed3));
  } else {
    c.occ = pin(gp(P.occ));
    c.nm_f = pin(gp(P.nm_f));
    c.visited = pin(gp(P.visited));
    c.cell2 = pin(gp(A.cell2));
    c.prevl = pin(gp(A.prevl));
    c.slots3 = pin(gp(A.slots3));
    c.closed3 = pin(gp(A.closed3));
  }
  c.open3 = pin(gp(A.open3));
  c.smask = pin(A.slots3_mask);
  c.N = pin(P.N);
  c.thr = pin(P.thr);
}

// ---------------------------------------------------------------- closed sets --------
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t slot_hash(uint32_t k) {
  k ^= k >> 16;
  k *= 0x7feb352du;
  k ^= k >> 15;
  k *= 0x846ca68bu;
  k ^= k >> 16;
  return k;
}

// unordered_set<Node3D>::insert(*it).first (HybridAStar.cpp:110): the existing record of
// the popped node's key, or a new copy of the popped open node.  *fresh tells which.
// The caller may issue the first probe early (closed3_probe) and pass it in.
__device__ __forceinline__ v2u closed3_probe(const SearchCtx& c, uint32_t key, uint32_t* h) {
  *h = slot_hash(key) & c.A->slots3_mask;
  return *(const GAS v2u*)&c.slots3[*h];
}
__device__ __forceinline__ int closed3_insert(SearchCtx& c, const Node3& n, bool* fresh, uint32_t h, v2u first) {
  const SlotArena& A = *c.A;
  const uint32_t gbits = (c.gen3 & SLOT3_GEN_MASK) << SLOT3_IDX_BITS;
  for (bool at_first = true;; at_first = false) {
    GAS v2u* s = (GAS v2u*)&c.slots3[h];
    const v2u sv = at_first ? first : *s;  // {key, gi}
    if ((sv.y & ~SLOT3_IDX_MASK) != gbits) {
      *fresh = true;
      if (c.n_closed3 >= A.closed3_cap) return NIL;
      const int idx = c.n_closed3++;
      Closed3 r;
      r.key = n.key;
      r.g = n.g;
      r.vmin = n.vmin;
      r.prev = n.prev;
      r.x = n.x;
      r.y = n.y;
      r.h = n.h;
      r.ci = (int)(n.cc >> 8);
      gstore(&c.closed3[idx], r);
      *s = v2u{n.key, gbits | (uint32_t)idx};
      return idx;
    }
    if (sv.x == n.key) {
      *fresh = false;
      return (int)(sv.y & SLOT3_IDX_MASK);
    }
    h = (h + 1) & c.smask;
  }
}

__device__ __forceinline__ bool closed3_contains(const SearchCtx& c, uint32_t key) {
  uint32_t h = slot_hash(key) & c.smask;
  const uint32_t gbits = (c.gen3 & SLOT3_GEN_MASK) << SLOT3_IDX_BITS;
  for (;;) {
    const v2u s = *(const GAS v2u*)&c.slots3[h];  // {key, gi}
    if ((s.y & ~SLOT3_IDX_MASK) != gbits) return false;
    if (s.x == key) return true;
    h = (h + 1) & c.smask;
  }
}

// next closed-set generation of this slot; when the 8-bit generation (SLOT3_GEN_MASK) wraps,
// the wave zeroes its hash table: every 255 searches, a pass over the whole table (several
// MiB for a 196k-pop arena: ~2 x max_pops slots of 8 B), amortised over those searches
__device__ __forceinline__ void closed3_next_gen(SearchCtx& c) {
  c.gen3 = (c.gen3 + 1) & SLOT3_GEN_MASK;
  if (c.gen3 == 0) {
    typedef int v4 __attribute__((ext_vector_type(4)));
    GAS v4* t = (GAS v4*)c.slots3;
    const size_t n4 = ((size_t)c.smask + 1) / 2;  // two 8-B slots per 16-B store
    for (size_t i = c.lane; i < n4; i += 64) t[i] = v4{0, 0, 0, 0};
    wave_lds_sync();
    c.gen3 = 1;
  }
}

// Resume of a parked search (SearchResult): the host copied the closed records into this
// arena; their hash slots are rebuilt here with the arena's next generation.  Lanes insert
// different keys concurrently: a slot is claimed by a compare-and-swap of its generation
// word, so every probe sequence stays contiguous (claims are never undone).
__device__ __forceinline__ void closed3_rebuild(SearchCtx& c, int n) {
  const uint32_t gbits = (c.gen3 & SLOT3_GEN_MASK) << SLOT3_IDX_BITS;
  GAS Slot3* t = c.slots3;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // after a generation-wrap zeroing of the table
  for (int i = c.lane; i < n; i += 64) {
    const uint32_t key = c.closed3[i].key;
    uint32_t h = slot_hash(key) & c.smask;
    uint32_t cur = __hip_atomic_load((uint32_t*)&t[h].gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      if ((cur & ~SLOT3_IDX_MASK) == gbits) {
        h = (h + 1) & c.smask;
        cur = __hip_atomic_load((uint32_t*)&t[h].gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      const uint32_t prev = atomicCAS((uint32_t*)&t[h].gi, cur, gbits | (uint32_t)i);
      if (prev == cur) {
        t[h].key = key;
        break;
      }
      cur = prev;
    }
  }
  // the wave's later plain loads of the table must see the claims and keys
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
  __builtin_amdgcn_wave_barrier();
}

// -------------------------------------------------------- holonomic A* (AStar.cpp) -----
// Each lazy A* search (AStar::find_path(int, int), AStar.cpp:100-113) keeps its open
// tree in LDS as compact nodes: {key, f} (8 B), the links {l, r} (16 bit each) and p
// (16 bit), and one colour bit per node, 16 B per node with the f-ordered ring, so that
// 8 search wavefronts fit a CU's 160 KiB LDS (2 per SIMD, the register budget).  Each
// node's g and prev link live in the HBM slot arena (`pvg`, 8 B per node: read together
// with the popped node's prev at the pop, written once per insert after the expansion);
// so do the closed records and the cell -> closed-record map, and every pop needs exactly
// one HBM round trip (the popped node's {prev, g}, its cell's closed state and the 8
// neighbour probes, all in flight together).  A search whose tree outgrows LDS is
// migrated once (same pool indices) to HBM nodes and continues there.  Both modes run
// the same templated loop.
//
// The layout is a compile-time configuration (AStarCfg): the node capacity of the LDS pool
// and where the {prev, g} pairs live.  The batch kernel's waves share a CU eight ways
// (NarrowA: 1024 nodes, pairs in the HBM arena); the latency kernel gives one search a CU's
// whole LDS (WideA: 2048 nodes, pairs in LDS too, no HBM round trip for them).
template <int CAP_, bool PVG_LDS_>
struct AStarCfg {
  static constexpr int CAP = CAP_;          // LDS open-tree nodes (index 0 = header)
  static constexpr bool PVG_LDS = PVG_LDS_;
  static_assert(CAP >= 128 && CAP <= 64 * 32 && (CAP & (CAP - 1)) == 0,
                "a power of two in 128..2048: one colour VGPR holds 32 nodes per lane");
};
using NarrowA = AStarCfg<ASTAR_LDS_CAP, false>;
using WideA = AStarCfg<2048, true>;

typedef int v2i __attribute__((ext_vector_type(2)));
struct NodeKF {
  uint32_t key;
  float f;
};
struct LinkLR {
  int16_t l, r;  // NIL = -1
};
template <class CF, bool = CF::PVG_LDS>
struct PvgPart {};  // {prev, g} pairs in the HBM arena (SlotArena::prevl)
template <class CF>
struct PvgPart<CF, true> {
  v2i pg[CF::CAP];  // {prev, g bits} per node, in LDS
};
template <class CF>
struct AStarLdsT : PvgPart<CF> {
  NodeKF kf[CF::CAP];
  LinkLR lr[CF::CAP];
  int16_t p[CF::CAP];
  int16_t ring[CF::CAP];  // live node indices in f order (a ring: rank r at ring[(head + r) % CAP])
};
static_assert(sizeof(AStarLdsT<NarrowA>) == 16 * NarrowA::CAP, "LDS node layout");
static_assert(sizeof(AStarLdsT<WideA>) == 24 * WideA::CAP, "LDS node layout");

#define LAS __attribute__((address_space(3)))
template <class T>
__device__ __forceinline__ LAS T* lp(T* p) {
  return (LAS T*)p;
}

// the compact LDS layout for RBT<>; g and prev (HBM) are read by the search loop itself.
// The colours are bits of one VGPR (lane j: nodes 32 j .. 32 j + 31, 1 = black): a colour
// read is one v_readlane, a colour write one masked VALU update, no LDS round trip.
template <class CF>
struct LdsAcc {
  static constexpr bool kPathWalk = false;
  LAS AStarLdsT<CF>* s;
  int lane;
  uint32_t cb;
  // every field is accessed through its own type (no type punning: with strict aliasing a
  // 16-bit store through an int* view would not be ordered against int loads)
  __device__ __forceinline__ int L(int x) const { return ufi(s->lr[x].l); }
  __device__ __forceinline__ int R(int x) const { return ufi(s->lr[x].r); }
  __device__ __forceinline__ int P(int x) const { return ufi(s->p[x]); }
  __device__ __forceinline__ int C(int x) const {
    return (int)(((uint32_t)__builtin_amdgcn_readlane((int)cb, x >> 5) >> (x & 31)) & 1u);
  }
  __device__ __forceinline__ void sL(int x, int v) {
    s->lr[x].l = (int16_t)v;
  }
  __device__ __forceinline__ void sR(int x, int v) {
    s->lr[x].r = (int16_t)v;
  }
  __device__ __forceinline__ void sP(int x, int v) {
    s->p[x] = (int16_t)v;
  }
  __device__ __forceinline__ void sC(int x, int v) {
    const uint32_t bit = 1u << (x & 31);
    const uint32_t nw = v == RB_BLACK ? (cb | bit) : (cb & ~bit);
    cb = lane == (x >> 5) ? nw : cb;
  }
  __device__ __forceinline__ uint32_t K(int x) const { return ufu(s->kf[x].key); }
  __device__ __forceinline__ float F(int x) const { return uff(s->kf[x].f); }
  __device__ __forceinline__ Quad quad(int x) const {
    const uint32_t k = s->kf[x].key;
    const float f = s->kf[x].f;
    const int l = s->lr[x].l, r = s->lr[x].r;
    Quad q;
    q.key = ufu(k);
    q.f = uff(f);
    q.l = ufi(l);
    q.r = ufi(r);
    return q;
  }
  __device__ __forceinline__ Quad quad_at(int x, int) const { return quad(x); }
  __device__ __forceinline__ void leaf(int x, int p) {
    s->lr[x].l = (int16_t)NIL;
    s->lr[x].r = (int16_t)NIL;
    s->p[x] = (int16_t)p;
    sC(x, RB_RED);
  }
  __device__ __forceinline__ void payload(int x, uint32_t key, float f, float g, int prev) {
    s->kf[x].key = key;
    s->kf[x].f = f;
    (void)g;     // pvg[x] = {prev, g} is stored by the caller after the expansion
    (void)prev;  // (see astar_loop_lds)
  }
};
// ---- f-ordered index of the LDS tree -------------------------------------------------
// The reference's open-set comparator keeps the tree's in-order sequence STRICTLY
// increasing in f (an insert whose in-order predecessor has an equal f, or the same cell,
// is dropped).  So while no node of the probed cell sits on the "wrong" side of the probe
// value, std::set::find / insert are decided by f ranks alone, independent of the tree
// shape: find(k, f) returns the first node with f' >= f when f' == f or it is the cell's
// own node; insert(k, f) attaches the new node between its rank neighbours (as the right
// child of the predecessor when that slot is free, else as the left child of the
// successor) unless the predecessor has f' == f or the same cell.  The wavefront answers
// those rank queries with a 2-level parallel search over a ring of node indices kept in f
// order (64 samples, then 16), instead of a ~10-level dependent tree walk.  The tree
// itself is still maintained exactly (link / rebalance / erase), and the rare shape-
// dependent cases (a node of the same cell with f' < probe f for find, f' > new f for
// insert, or several nodes of that cell) fall back to the tree walks.
struct Ring {
  int head, n;
};
struct RankOut {
  int r;        // #(live f < v)
  int at;       // node at rank r (first with f >= v), NIL if r == n
  float at_f;
  int pred;     // node at rank r - 1, NIL if r == 0
};

// Level 1 samples every SR-th rank (64 lanes cover CAP ranks, SR = CAP / 64); level 2 resolves
// the SR ranks of one bucket per value (lanes [0, SR) for value A, [SR, 2 SR) for value B).
template <int SR>
__device__ __forceinline__ void rank_out(RankOut& O, int b, int cnt, int off, int n, int i1, float f1, int i2,
                                         float f2) {
  auto rl_i = [](int v, int l) { return __builtin_amdgcn_readlane(v, l); };
  auto rl_f = [](float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); };
  if (b == 0) {
    O.r = 0;
    O.pred = NIL;
    O.at = n > 0 ? rl_i(i1, 0) : NIL;
    O.at_f = n > 0 ? rl_f(f1, 0) : 0.0f;
    return;
  }
  O.r = (b - 1) * SR + cnt;
  O.pred = rl_i(i2, off + cnt - 1);
  if (O.r >= n) {
    O.at = NIL;
    O.at_f = 0.0f;
  } else if (cnt < SR) {
    O.at = rl_i(i2, off + cnt);
    O.at_f = rl_f(f2, off + cnt);
  } else {
    O.at = rl_i(i1, b);
    O.at_f = rl_f(f1, b);
  }
}

template <class CF>
__device__ __forceinline__ void rank2(const AStarLdsT<CF>& L, const Ring& rg, float vA, float vB, int lane, RankOut& A,
                                      RankOut& B) {
  constexpr int SR = CF::CAP / 64;
  constexpr int M = CF::CAP - 1;
  constexpr uint64_t SMASK = (SR == 32) ? 0xffffffffull : ((1ull << SR) - 1);
  const int n = rg.n;
  const int s_r = lane * SR;
  const bool h1 = s_r < n;
  const int i1 = (int)L.ring[(rg.head + s_r) & M] & M;  // unconditional loads, masked use
  const float f1 = L.kf[i1].f;
  const int bA = __popcll(__ballot(h1 && f1 < vA)), bB = __popcll(__ballot(h1 && f1 < vB));
  const bool forA = lane < SR;
  const int bb = forA ? bA : bB;
  const int sub = lane & (SR - 1);
  const int r2 = (bb - 1) * SR + sub;
  const bool h2 = lane < 2 * SR && bb > 0 && r2 < n;
  const int i2 = (int)L.ring[(rg.head + r2) & M] & M;
  const float f2 = L.kf[i2].f;
  const uint64_t m2 = __ballot(h2 && f2 < (forA ? vA : vB));
  const int cA = __popcll(m2 & SMASK), cB = __popcll((m2 >> SR) & SMASK);
  // lanes of level 2 hold ranks base..base+SR-1; rank base+SR is level-1 sample lane b
  rank_out<SR>(A, bA, cA, 0, n, i1, f1, i2, f2);
  rank_out<SR>(B, bB, cB, SR, n, i1, f1, i2, f2);
}

// Shift `cnt` consecutive ring entries by one slot (dir = -1: entries at ring offsets
// [from, from + cnt) move to [from - 1, ...); dir = +1: they move to [from + 1, ...)).  All
// of a lane's loads (one per 64 entries, at most A_CAP / 2 entries: the shorter side) are
// issued before its stores, so the shift costs one LDS round trip instead of one per 64
// entries.  Positions are ring offsets relative to `head` (masked by A_CAP - 1).
// EXACT: the shift has exactly NCH chunks (chunks 0 .. NCH - 2 are full, only the last may be
// partial); else at most NCH (each entry tested against cnt).
template <class CF, int NCH, bool EXACT>
__device__ __forceinline__ void ring_shift_n(AStarLdsT<CF>& L, int head, int from, int cnt, int dir, int lane) {
  constexpr int M = CF::CAP - 1;
  int16_t v[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int i = c * 64 + lane;
    v[c] = 0;
    if ((EXACT && c < NCH - 1) || i < cnt) v[c] = L.ring[(head + from + i) & M];
  }
  wave_lds_sync();
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int i = c * 64 + lane;
    if ((EXACT && c < NCH - 1) || i < cnt) L.ring[(head + from + i + dir) & M] = v[c];
  }
  wave_lds_sync();
}
template <class CF>
__device__ __forceinline__ void ring_shift(AStarLdsT<CF>& L, int head, int from, int cnt, int dir, int lane) {
  constexpr int RING_CH = CF::CAP / 2 / 64;  // chunks of 64 entries in the shorter side
  static_assert(RING_CH >= 4, "ring_shift's specialised chunk counts");
  // the chunk count is wave-uniform: one straight-line copy per count (the short shifts of a
  // small open set do not test the chunks they do not have)
  if (HASTAR_LIKELY(cnt <= 64)) {  // the common short shift near an end of the ring
    ring_shift_n<CF, 1, true>(L, head, from, cnt, dir, lane);
    return;
  }
  switch ((cnt + 63) >> 6) {
    case 1: ring_shift_n<CF, 1, true>(L, head, from, cnt, dir, lane); break;
    case 2: ring_shift_n<CF, 2, true>(L, head, from, cnt, dir, lane); break;
    case 3: ring_shift_n<CF, 3, true>(L, head, from, cnt, dir, lane); break;
    case 4: ring_shift_n<CF, 4, true>(L, head, from, cnt, dir, lane); break;
    default: ring_shift_n<CF, RING_CH, false>(L, head, from, cnt, dir, lane); break;
  }
}

// ring insert of node x at rank r (shifts the shorter side by one)
template <class CF>
__device__ __forceinline__ void ring_insert(AStarLdsT<CF>& L, Ring& rg, int r, int x, int lane) {
  constexpr int M = CF::CAP - 1;
  if (r < rg.n - r) {  // ranks [0, r) move one slot down, head - 1
    if (r > 0) ring_shift(L, rg.head, 0, r, -1, lane);
    rg.head = (rg.head - 1) & M;
  } else {  // ranks [r, n) move one slot up
    if (rg.n > r) ring_shift(L, rg.head, r, rg.n - r, +1, lane);
  }
  if (lane == 0) L.ring[(rg.head + r) & M] = (int16_t)x;
  rg.n++;
  wave_lds_sync();
}

// ring erase of the node at rank r
template <class CF>
__device__ __forceinline__ void ring_erase(AStarLdsT<CF>& L, Ring& rg, int r, int lane) {
  constexpr int M = CF::CAP - 1;
  if (r < rg.n - 1 - r) {  // ranks [0, r) move one slot up, head + 1
    if (r > 0) ring_shift(L, rg.head, 0, r, +1, lane);
    rg.head = (rg.head + 1) & M;
  } else {  // ranks (r, n) move one slot down
    if (rg.n - 1 > r) ring_shift(L, rg.head, r + 1, rg.n - 1 - r, -1, lane);
  }
  rg.n--;
}

// nodes of cell `key` among the pool's used slots: cnt 0, 1 (idx, f) or 2 (= several)
struct SameCell {
  int cnt, idx;
  float f;
};
template <class CF>
__device__ __forceinline__ SameCell same_cell(const AStarLdsT<CF>& L, int used, uint32_t key, int lane) {
  // all loads unconditional (in-bounds by construction) so they issue back to back
  constexpr int Q = CF::CAP / 64;
  uint32_t kk[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) kk[q] = L.kf[lane + 64 * q].key;
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < Q; ++q) m |= (uint32_t)((lane + 64 * q < used) & (kk[q] == key)) << q;
  const uint64_t any = __ballot(m != 0);
  SameCell sc;
  sc.cnt = 0;
  sc.idx = NIL;
  sc.f = 0.0f;
  if (any == 0) return sc;
  if (__popcll(any) > 1) {
    sc.cnt = 2;
    return sc;
  }
  const int ln = __ffsll((unsigned long long)any) - 1;
  const uint32_t mm = (uint32_t)__builtin_amdgcn_readlane((int)m, ln);
  if (__popc(mm) > 1) {
    sc.cnt = 2;
    return sc;
  }
  sc.cnt = 1;
  sc.idx = ln + 64 * (__ffs(mm) - 1);
  sc.f = uff(L.kf[sc.idx].f);
  return sc;
}

// HBM layout (Node2, 32-bit links, prev in the node)
struct HbmAcc : AosAcc<Node2, GAS Node2*> {
  __device__ __forceinline__ float G(int x) const { return t[x].g; }
  __device__ __forceinline__ int PV(int x) const { return t[x].prev; }
  __device__ __forceinline__ void payload(int x, uint32_t key, float f, float g, int prev) {
    t[x].key = key;
    t[x].f = f;
    t[x].g = g;
    t[x].prev = prev;
  }
};

// AStar::update_visted + Grid2D::update_costs (AStar.cpp:209-218, Grid2D.cpp:219-227):
// the prev chain of closed records, which are the cells' own records
__device__ __forceinline__ void memoise(SearchCtx& c, float total, int from) {
  const GAS Cell2* cells = c.cell2;
  const uint32_t NN = (uint32_t)c.N * (uint32_t)c.N;
  for (int i = from; i != NIL && (uint32_t)i < NN;) {  // (the bound only guards a corrupted chain)
    const Cell2 r = gload(&cells[i]);
    GAS uint32_t* vw = &c.visited[(uint32_t)i >> 5];
    *vw = *vw | (1u << (i & 31));  // one wave owns the planner: a plain read-modify-write
    c.nm_f[i] = total - r.g;
    i = r.prev;
  }
}

template <class Tree>
__device__ __forceinline__ bool insert2(SearchCtx& c, Tree& tr, int cap, uint32_t key, float f, float g, int prev) {
  bool left;
  const int pos = tr.insert_pos(key, f, &left);
  if (pos == -2) return true;  // equal-f "duplicate": dropped like std::set::insert
  const int n = tpool_alloc(tr, c.ps2, cap);
  if (n == NIL) return false;
  tr.payload(n, key, f, g, prev);
  tr.link(left, n, pos);
  return true;
}

// The body of AStar::a_star_search (AStar.cpp:118-186).  G = false: LDS tree, returns
// false (without popping) when the next pop could overflow the LDS pool.  Returns true
// when the search finished; *result = cost-to-goal or FLT_MAX.
template <bool G, class Tree>
__device__ __forceinline__ bool astar_loop(SearchCtx& c, Tree& tr, int adx, int ady, float acost, float* result) {
  const PlannerDev& P = *c.P;
  const SlotArena& A = *c.A;
  const int lane = c.lane;
  const int nact = P.diag ? 8 : 4;
  GAS Cell2* cells = c.cell2;
  static_assert(G, "the LDS mode is astar_loop_lds");
  const int cap = A.open2_cap < P.astar_cap ? A.open2_cap : P.astar_cap;  // the planner's max_astar_nodes
  while (!tr.empty()) {
    STAMP_T t_pop = STAMP_NOW();
    const int b = tr.begin();
    const Quad top = tr.quad(b);
    const float top_g = uff(tr.G(b));
    const int tx = (int)(top.key >> 16), ty = (int)(top.key & 0xffffu);
    const uint32_t tcell = (uint32_t)tx * (uint32_t)c.N + (uint32_t)ty;
    // one HBM round trip: the popped cell's closed state and prev link, and the
    // neighbour probes (bounds, occupancy, memo flag, node-map f, closed membership —
    // loop-invariant during this expansion; Grid2D::get_neighbors, Grid2D.cpp:72-96)
    const Cell2 tc = gload(&cells[tcell]);
    const int tprev = ufi(tr.PV(b));
    const int ni = tx + adx, nj = ty + ady;
    bool valid = false, vis = false, closed = false;
    float nf = 0.0f;
    if (lane < nact && ni > -1 && ni < c.N && nj > -1 && nj < c.N) {
      const uint32_t cell = (uint32_t)ni * (uint32_t)c.N + (uint32_t)nj;
      const float occv = c.occ[cell];
      const uint32_t visw = c.visited[cell >> 5];
      nf = c.nm_f[cell];
      const uint32_t cg = cells[cell].cgen;
      valid = occv < c.thr;
      vis = valid && ((visw >> (cell & 31)) & 1u);
      closed = valid && cg == c.gen2;
    }
    tr.unlink(b);
    tpool_free(tr, c.ps2, b);
    // unordered_set::insert(*it).first (AStar.cpp:130): a duplicate expands the OLD record
    // (the cell's record; the popped node is of the same cell)
    const int ci = (int)tcell;
    float g0;
    if (ufu(tc.cgen) == c.gen2) {
      g0 = uff(tc.g);
    } else {
      g0 = top_g;
      Cell2 rec;
      rec.cgen = c.gen2;
      rec.g = top_g;
      rec.prev = tprev;
      rec.oinfo = tc.oinfo;
      gstore(&cells[tcell], rec);
    }
    c.apops++;
    if (G) c.apops_g++;
    if (HASTAR_UNLIKELY(tx == P.goal_cx && ty == P.goal_cy)) {
      const float fgoal = g0 + euclid_h(P, tx, ty);  // the record's f (Node2D: f = g + h)
      if (c.cost_only) memoise(c, fgoal, ci);
      *result = fgoal;
      return true;
    }
    const uint64_t vmask = __ballot(valid), vismask = c.cost_only ? __ballot(vis) : 0ull, cmask = __ballot(closed);
    if (!G) STAMP_ADD(8, t_pop);
    for (int k = 0; k < nact; ++k) {
      if (!((vmask >> k) & 1ull)) continue;
      const float kcost = rl_f(acost, k);
      if (HASTAR_UNLIKELY((vismask >> k) & 1ull)) {
        const float tot = rl_f(nf, k) + g0 + kcost;
        STAMP_T t_m = STAMP_NOW();
        memoise(c, tot, ci);
        STAMP_ADD(12, t_m);
        *result = tot;
        return true;
      }
      if ((cmask >> k) & 1ull) continue;
      const int ki = rl_i(ni, k), kj = rl_i(nj, k);
      const uint32_t key = ((uint32_t)ki << 16) | (uint32_t)kj;
      const float fprobe = rl_f(nf, k);  // stale _node_map f, as the reference reads it
      STAMP_T t_f = STAMP_NOW();
      const int hit = tr.find(key, fprobe);
      if (!G) STAMP_ADD(9, t_f);
      const float gn = g0 + kcost;
      if (hit == 0) {
        const float fn = gn + euclid_h(P, ki, kj);
        c.nm_f[(size_t)ki * c.N + kj] = fn;  // Node2D::set_accumulated_cost
        STAMP_T t_i = STAMP_NOW();
        if (!insert2(c, tr, cap, key, fn, gn, ci)) { c.status = -75; *result = FLT_MAX; return true; }
        if (!G) STAMP_ADD(10, t_i);
      } else if (gn < tr.G(hit)) {
        STAMP_T t_u = STAMP_NOW();
        tr.unlink(hit);
        tpool_free(tr, c.ps2, hit);
        if (!G) STAMP_ADD(11, t_u);
        const float fn = gn + euclid_h(P, ki, kj);
        c.nm_f[(size_t)ki * c.N + kj] = fn;
        if (!insert2(c, tr, cap, key, fn, gn, ci)) { c.status = -75; *result = FLT_MAX; return true; }
      }
    }
    wave_lds_sync();
  }
  *result = FLT_MAX;
  return true;
}

// insert (AStar.cpp:172-183) into the LDS tree: rank-decided unless shape-dependent
// The LDS pool's free list is threaded through the dead nodes' f field (key 0xffffffff marks
// them), not through their links: a node freed while its erase is still in the log keeps the
// links the replay's unlink reads.
template <class CF>
__device__ __forceinline__ void free_lds(SearchCtx& c, RBT<LdsAcc<CF>>& tr, int x) {
  tr.s->kf[x].key = 0xffffffffu;  // dead: never matches a cell
  tr.s->kf[x].f = __int_as_float(c.ps2.free);
  c.ps2.free = x;
}
template <class CF>
__device__ __forceinline__ int alloc_lds(SearchCtx& c, RBT<LdsAcc<CF>>& tr) {
  if (c.ps2.free != NIL) {
    const int i = c.ps2.free;
    c.ps2.free = __builtin_amdgcn_readfirstlane(__float_as_int(tr.s->kf[i].f));
    return i;
  }
  if (HASTAR_UNLIKELY(c.ps2.next >= CF::CAP)) return NIL;
  return c.ps2.next++;
}

// ---- deferred inner tree ------------------------------------------------------------
// An inner search keeps only its f-ordered ring while no shape-dependent event has happened:
// the pop takes the ring's first node (the tree's leftmost), and an insert's position comes
// from its rank neighbours, so the red-black links are not needed.  Each tree operation is
// logged instead ({node, insert flag} and its rank neighbours {pred, at}; the pop's and the
// expansion's entries in lanes 0.., stored to the arena's open2 area at the end of the pop).
// At an event that needs the tree (a find or insert walk, a migration to HBM, or a full log)
// the log is replayed into the tree as it stood at the last replay (empty at the search's
// start): the same libstdc++ link / erase calls in the same order give the same shape, so
// results are identical.  Then logging goes on.  Searches that end without an event never
// build their tree; the others build it only at their events.
struct Pend {
  uint32_t lo, hi;  // lane j: entry j of this pop (lo = node | insert << 31, hi = pred | at << 16)
  int n;            // entries pending (wave-uniform, in a VGPR)
  int logn;         // entries in the log
};
// (deferral is always on: a replay leaves logn = 0 and logging goes on, so the tree-mode
// branches behind pend_on are never taken and compile away)
__device__ __forceinline__ bool pend_on(const Pend&) { return true; }
__device__ __forceinline__ void pend_add(Pend& pd, int lane, int x, bool ins, int pred, int at) {
  const bool me = lane == pd.n;
  pd.lo = me ? ((uint32_t)x | (ins ? 0x80000000u : 0u)) : pd.lo;
  pd.hi = me ? (((uint32_t)pred & 0xffffu) | ((uint32_t)at << 16)) : pd.hi;
  pd.n += 1;
}
template <class CF>
__device__ __forceinline__ void pend_replay(SearchCtx& c, RBT<LdsAcc<CF>>& tr, AStarLdsT<CF>& L, Pend& pd) {
  auto apply = [&](uint32_t lo, uint32_t hi) {
    const int x = (int)(lo & 0xffffu);
    if (lo >> 31) {
      const int pred = (int)(int16_t)(hi & 0xffffu), at = (int)(int16_t)(hi >> 16);
      int parent;
      bool left;
      if (pred == NIL && at == NIL) {  // into the empty tree
        parent = 0;
        left = true;
      } else if (pred == NIL) {
        parent = at;
        left = true;
      } else if (at == NIL || tr.R(pred) == NIL) {
        parent = pred;
        left = false;
      } else {
        parent = at;
        left = true;
      }
      tr.link(left, x, parent);
    } else {
      tr.unlink(x);
    }
  };
  const int lane = c.lane;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's log stores are in L2
  const int logn = __builtin_amdgcn_readfirstlane(pd.logn);
  GAS uint32_t* lg = (GAS uint32_t*)gp(c.A->open2);
  for (int base = 0; base < logn; base += 64) {
    uint32_t lo = 0, hi = 0;
    if (base + lane < logn) {  // (L1-bypassing loads: the lines were written since any earlier read)
      lo = __hip_atomic_load((uint32_t*)&lg[2 * (base + lane)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      hi = __hip_atomic_load((uint32_t*)&lg[2 * (base + lane) + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int cnt = min(64, logn - base);
    for (int j = 0; j < cnt; ++j)
      apply((uint32_t)__builtin_amdgcn_readlane((int)lo, j), (uint32_t)__builtin_amdgcn_readlane((int)hi, j));
  }
  const int np = __builtin_amdgcn_readfirstlane(pd.n);
  for (int j = 0; j < np; ++j)
    apply((uint32_t)__builtin_amdgcn_readlane((int)pd.lo, j), (uint32_t)__builtin_amdgcn_readlane((int)pd.hi, j));
  wave_lds_sync();
  pd.logn = 0;  // the tree is current; later operations are logged again
  pd.n = 0;
}

template <class CF>
__device__ __forceinline__ bool insert_lds(SearchCtx& c, RBT<LdsAcc<CF>>& tr, AStarLdsT<CF>& L, Ring& rg, uint32_t key,
                                           float fn, float gn, int prev, const SameCell& sc, const RankOut& rb,
                                           int* node_out, Pend& pd) {
  *node_out = NIL;
  int parent = 0;
  bool left = true;
  bool logged = false;
  if (HASTAR_UNLIKELY(sc.cnt >= 2 || (sc.cnt == 1 && sc.f > fn))) {  // a node of this cell lies right of fn
    if (pend_on(pd)) pend_replay(c, tr, L, pd);  // the walk needs the tree
    parent = tr.insert_pos(key, fn, &left);
    if (parent == -2) return true;
  } else {
    if (HASTAR_UNLIKELY((rb.at != NIL && rb.at_f == fn) || (rb.pred != NIL && rb.pred == sc.idx))) return true;  // dropped
    if (pend_on(pd)) {
      logged = true;  // its place is its rank neighbours: linked when the log is replayed
    } else if (rg.n == 0) {
      parent = 0;
      left = true;
    } else if (rb.pred == NIL) {
      parent = rb.at;
      left = true;
    } else if (rb.at == NIL || tr.R(rb.pred) == NIL) {
      parent = rb.pred;
      left = false;
    } else {
      parent = rb.at;
      left = true;
    }
  }
  const int n = alloc_lds(c, tr);
  if (HASTAR_UNLIKELY(n == NIL)) return false;
  tr.payload(n, key, fn, gn, prev);
  STAMP_T t_l = STAMP_NOW();
  if (logged) pend_add(pd, c.lane, n, true, rg.n == 0 ? NIL : rb.pred, rg.n == 0 ? NIL : rb.at);
  else tr.link(left, n, parent);
  STAMP_ADD(25, t_l);
  STAMP_T t_r = STAMP_NOW();
  ring_insert(L, rg, rb.r, n, c.lane);
  STAMP_ADD(30, t_r);
  *node_out = n;
  return true;
}

// The record of a cell whose node was just inserted into the open tree (one 16-B store): not
// closed (cgen != this search's generation), the node's g and prev link, and the hint.
__device__ __forceinline__ void open_cell(GAS Cell2* cells, uint32_t cell, uint32_t open_cgen, float g, int prev,
                                          uint32_t gen2, uint32_t hint) {
  Cell2 r;
  r.cgen = open_cgen;
  r.g = g;
  r.prev = prev;
  r.oinfo = ((gen2 & CELL2_OGEN_MASK) << CELL2_OGEN_SHIFT) | hint;
  gstore(&cells[cell], r);
}

// g of open node `hit` (the find result for neighbour k): a node inserted earlier in this
// expansion (its {prev, g} store is still pending in the inserting lane), lane k's hinted node
// when it is still that cell's node (own: its g is the cell record's, loaded with the neighbour
// probes; a hinted index that now holds another cell's node has a g of its own), or the node's
// {prev, g} pair.
// {prev, g} of LDS-tree node x: in LDS (WideA) or in the HBM arena (NarrowA)
template <class CF>
__device__ __forceinline__ v2i pvg_load(const SearchCtx& c, AStarLdsT<CF>& L, int x) {
  if constexpr (CF::PVG_LDS) return *lp(&L.pg[x & (CF::CAP - 1)]);
  else return *(const GAS v2i*)&c.prevl[2 * (x & (CF::CAP - 1))];
}
template <class CF>
__device__ __forceinline__ void pvg_store(const SearchCtx& c, AStarLdsT<CF>& L, int x, int prev, float g) {
  if constexpr (CF::PVG_LDS) *lp(&L.pg[x & (CF::CAP - 1)]) = v2i{prev, __float_as_int(g)};
  else *(GAS v2i*)&c.prevl[2 * (x & (CF::CAP - 1))] = v2i{prev, __float_as_int(g)};
}

template <class CF>
__device__ __forceinline__ float hit_g(const SearchCtx& c, AStarLdsT<CF>& L, int hit, int k, int hy, float hg,
                                       bool own, bool st_pv, int st_node, float st_g) {
  const uint64_t pend = __ballot(st_pv && st_node == hit);
  if (pend) return rl_f(st_g, (int)__ffsll((unsigned long long)pend) - 1);
  if (own && rl_i(hy, k) == hit) return rl_f(hg, k);  // not reused in this expansion (else pending)
  return uff(__int_as_float(pvg_load(c, L, hit).y));
}

// AStar::a_star_search (AStar.cpp:118-186) on the LDS tree.  Returns false (without
// popping) when the next pop could overflow the LDS pool; true when the search finished
// (*result = cost-to-goal or FLT_MAX).
template <class CF>
__device__ __forceinline__ bool astar_loop_lds(SearchCtx& c, RBT<LdsAcc<CF>>& tr, AStarLdsT<CF>& L, Ring& rg, int adx,
                                               int ady, float acost, float* result, Pend& pd) {
  const PlannerDev& P = *c.P;
  const int lane = c.lane;
  const int nact = P.diag ? 8 : 4;
  GAS Cell2* cells = c.cell2;
  // an open (not closed) cell's record holds its hinted node's g and prev link, written with
  // the hint; cgen = any value but this search's generation
  const uint32_t open_cgen = c.gen2 - 1u;
  // migrate before a pop that could take the pool past the LDS capacity or the arena's HBM
  // tree (the migration copies every index in use into A.open2, and max_astar_nodes bounds the
  // inner search in both modes and on both kernels alike)
  const int acap = c.A->open2_cap < P.astar_cap ? c.A->open2_cap : P.astar_cap;
  const int lim = CF::CAP < acap ? CF::CAP : acap;
  // the log's capacity in 8-B entries (the open2 area, unused until a migration), less one
  // pop's entries (1 + 2 per neighbour)
  const int log_lim = c.A->open2_cap * (int)(sizeof(Node2) / 8) - (1 + 2 * 8);
  while (rg.n > 0) {
    if (HASTAR_UNLIKELY(c.ps2.next + 8 > lim)) return false;
    if (pend_on(pd) && HASTAR_UNLIKELY(__builtin_amdgcn_readfirstlane(pd.logn) > log_lim)) pend_replay(c, tr, L, pd);
    STAMP_T t_pop = STAMP_NOW();
    const int b = pend_on(pd) ? ((int)L.ring[rg.head] & (CF::CAP - 1)) : tr.begin();
    const Quad top = tr.quad(b);
    const int tx = (int)(top.key >> 16), ty = (int)(top.key & 0xffffu);
    const uint32_t tcell = (uint32_t)tx * (uint32_t)c.N + (uint32_t)ty;
    const v2i tpg = pvg_load(c, L, b);  // the popped node's {prev, g}
    const Cell2 tc = gload(&cells[tcell]);
    const int ni = tx + adx, nj = ty + ady;
    // the neighbour probes are only issued here; the popped node leaves the LDS tree while they
    // are in flight (the erase needs none of them), and they are consumed after it
    const bool inb = lane < nact && ni > -1 && ni < c.N && nj > -1 && nj < c.N;
    const uint32_t cell = inb ? (uint32_t)ni * (uint32_t)c.N + (uint32_t)nj : 0u;
    float occv = 0.0f, nf = 0.0f;
    uint32_t visw = 0u;
    Cell2 cr{};
    if (inb) {
      occv = c.occ[cell];
      visw = c.visited[cell >> 5];
      nf = c.nm_f[cell];
      cr = gload(&cells[cell]);
    }
    STAMP_T t_u = STAMP_NOW();
    if (pend_on(pd)) pend_add(pd, lane, b, false, NIL, NIL);
    else tr.unlink(b);
    STAMP_ADD(24, t_u);
    free_lds(c, tr, b);
    ring_erase(L, rg, 0, lane);
    // consume every probe before the first store of this pop, so that no later register
    // reuse has to wait on a store (vmcnt counts loads and stores in issue order)
    const bool valid = inb && occv < c.thr;
    const bool vis = valid && ((visw >> (cell & 31)) & 1u);
    const bool closed = valid && cr.cgen == c.gen2;
    // this lane's cell: last open node (| dup << 16), or none; hg = that node's g (the open
    // cell's record)
    const uint32_t ohint = (inb && (cr.oinfo >> CELL2_OGEN_SHIFT) == (c.gen2 & CELL2_OGEN_MASK))
                               ? (cr.oinfo & CELL2_HINT_MASK) : 0xffffffffu;
    const float hg = inb ? cr.g : 0.0f;
    const uint64_t vmask = __ballot(valid), vismask = c.cost_only ? __ballot(vis) : 0ull, cmask = __ballot(closed);
    nf = __builtin_amdgcn_readfirstlane(0) + nf;  // keep nf live in a VGPR (no-op)
    const int tprev = ufi(tpg.x);
    const float top_g = uff(__int_as_float(tpg.y));
    // this lane's hinted open node (the node a find of this cell usually returns); its g came
    // with the probe (hg), and a node's g never changes while it is open
    const int hy = (ohint != 0xffffffffu && !((ohint >> 16) & 1u)) ? (int)(ohint & 0xffffu) : NIL;
    // that node's {key, f} for every lane in one LDS round trip (the popped node is already
    // dead).  A node's key and f do not change while it lives, and no node gets a neighbour's
    // cell before that neighbour's own insert, so these stay exact for the whole expansion
    // unless a node is freed in it (a replaced find hit: then `freed` and the loop re-reads)
    uint32_t hkey = 0xffffffffu;
    float hf = 0.0f;
    if (hy != NIL) {
      hkey = L.kf[hy].key;
      hf = L.kf[hy].f;
    }
    bool freed = false;
    const int ci = (int)tcell;  // closed record = the cell's record
    float g0;
    if (ufu(tc.cgen) == c.gen2) {
      g0 = uff(tc.g);
    } else {
      g0 = top_g;
      Cell2 rec;
      rec.cgen = c.gen2;
      rec.g = top_g;
      rec.prev = tprev;
      rec.oinfo = tc.oinfo;
      gstore(&cells[tcell], rec);
    }
    c.apops++;
    if (tx == P.goal_cx && ty == P.goal_cy) {
      const float fgoal = g0 + euclid_h(P, tx, ty);  // the record's f (Node2D: f = g + h)
      if (c.cost_only) memoise(c, fgoal, ci);
      *result = fgoal;
      return true;
    }
    STAMP_ADD(8, t_pop);
    STAMP_T t_pre = STAMP_NOW();
    // every neighbour's key, g and f (AStar.cpp:160-176) in its own lane, in the reference's
    // float order (g0 + cost, then + h): the loop below reads them instead of computing them
    const uint32_t key_l = ((uint32_t)ni << 16) | ((uint32_t)nj & 0xffffu);
    const float gn_l = g0 + acost;
    const float fn_l = gn_l + euclid_h(P, ni, nj);
    // The expansion's HBM stores (node-map f of inserted cells, prev links of new nodes) are
    // collected in lane k and issued together after the loop: a global store inside the
    // loop would make every later register reuse wait for its completion (vmcnt).
    uint32_t st_cell = 0, st_hint = 0;
    float st_f = 0.0f, st_g = 0.0f;
    int st_node = NIL;
    bool st_on = false, st_pv = false;  // st_pv: pvg[st_node] = {ci, st_g} is still due
    STAMP_ADD(33, t_pre);
    STAMP_T t_nl = STAMP_NOW();
    for (int k = 0; k < nact; ++k) {
      if (!((vmask >> k) & 1ull)) continue;
      const float kcost = rl_f(acost, k);
      if ((vismask >> k) & 1ull) {
        const float tot = rl_f(nf, k) + g0 + kcost;
        if (st_on) {  // this expansion's earlier node-map writes happen before the return
          c.nm_f[st_cell] = st_f;
          if (st_node != NIL) {
            if (st_pv) pvg_store(c, L, st_node, ci, st_g);
            open_cell(cells, st_cell, open_cgen, st_g, ci, c.gen2, st_hint);
          }
        }
        STAMP_T t_m = STAMP_NOW();
        memoise(c, tot, ci);
        STAMP_ADD(12, t_m);
        *result = tot;
        return true;
      }
      if ((cmask >> k) & 1ull) continue;
      const int ki = rl_i(ni, k), kj = rl_i(nj, k);
      const uint32_t key = ufu((uint32_t)__builtin_amdgcn_readlane((int)key_l, k));
      const float fprobe = rl_f(nf, k);  // stale _node_map f, as the reference reads it
      const float gn = rl_f(gn_l, k);    // g0 + kcost
      const float fn = rl_f(fn_l, k);    // gn + euclid_h(ki, kj)
      STAMP_T t_f = STAMP_NOW();
      // nodes of this cell in the open tree: from the cell's hint (its last inserted node;
      // exact unless a duplicate was ever inserted in this search, then scan the pool)
      const uint32_t hint = ufu((uint32_t)__builtin_amdgcn_readlane((int)ohint, k));
      bool dup = false;
      SameCell sc{0, NIL, 0.0f};
      if (hint != 0xffffffffu) {
        dup = (hint >> 16) & 1u;
        if (HASTAR_UNLIKELY(dup)) {
          sc = same_cell(L, c.ps2.next, key, lane);
        } else {
          const int y = (int)(hint & 0xffffu);  // = lane k's hy
          if (!freed) {
            if (ufu((uint32_t)__builtin_amdgcn_readlane((int)hkey, k)) == key) sc = SameCell{1, y, rl_f(hf, k)};
          } else if (ufu(L.kf[y].key) == key) {
            sc = SameCell{1, y, uff(L.kf[y].f)};
          }
        }
      }
      RankOut ra, rb;
      int hit = 0, hit_rank = -1;
      if (sc.cnt == 1 && sc.f == fprobe) {
        // the cell's only open node carries the probed f: the in-order f sequence is strictly
        // increasing, so every node left of it fails the lower_bound predicate and it passes
        // (equal key): find returns it whatever the tree shape, no rank query needed
        hit = sc.idx;
      } else {
        rank2(L, rg, fprobe, fn, lane, ra, rb);
        if (HASTAR_UNLIKELY(sc.cnt >= 2 || (sc.cnt == 1 && sc.f < fprobe))) {
          if (pend_on(pd)) pend_replay(c, tr, L, pd);
          hit = tr.find(key, fprobe);  // shape-dependent: the exact tree walk
        } else if (ra.at != NIL && (ra.at_f == fprobe || ra.at == sc.idx)) {
          hit = ra.at;
          hit_rank = ra.r;
        }
      }
      STAMP_ADD(9, t_f);
      if (HASTAR_LIKELY(hit == 0)) {
        STAMP_T t_i = STAMP_NOW();
        int nn;
        if (HASTAR_UNLIKELY(!insert_lds(c, tr, L, rg, key, fn, gn, ci, sc, rb, &nn, pd))) { c.status = -75; *result = FLT_MAX; return true; }
        if (lane == k) {  // Node2D::set_accumulated_cost; the cell's nm_f is written even
          st_on = true;   // when the insert is dropped (AStar.cpp:172-183)
          st_cell = (uint32_t)ki * (uint32_t)c.N + (uint32_t)kj;
          st_f = fn;
          st_g = gn;
          st_node = nn;
          st_pv = nn != NIL;
          st_hint = nn == NIL ? ohint : ((uint32_t)nn | (uint32_t)(dup || sc.cnt > 0) << 16);
        }
        STAMP_ADD(10, t_i);
      } else if (STAMP_T t_rp = STAMP_NOW(); gn < hit_g(c, L, hit, k, hy, hg, sc.cnt == 1 && sc.idx == hit, st_pv, st_node, st_g)) {
        STAMP_T t_u = STAMP_NOW();
        if (hit_rank < 0) {
          const float hf = tr.F(hit);
          RankOut h1, h2;
          rank2(L, rg, hf, hf, lane, h1, h2);
          hit_rank = h1.r;
        }
        if (pend_on(pd)) pend_add(pd, lane, hit, false, NIL, NIL);
        else tr.unlink(hit);
        free_lds(c, tr, hit);
        freed = true;
        ring_erase(L, rg, hit_rank, lane);
        if (st_node == hit) st_pv = false;  // a node inserted earlier in this expansion is gone
        STAMP_ADD(11, t_u);
        if (dup) sc = same_cell(L, c.ps2.next, key, lane);
        else if (hit == sc.idx) sc = SameCell{0, NIL, 0.0f};
        RankOut r1;
        rank2(L, rg, fn, fn, lane, r1, rb);
        int nn;
        if (!insert_lds(c, tr, L, rg, key, fn, gn, ci, sc, rb, &nn, pd)) { c.status = -75; *result = FLT_MAX; return true; }
        if (lane == k) {
          st_on = true;
          st_cell = (uint32_t)ki * (uint32_t)c.N + (uint32_t)kj;
          st_f = fn;
          st_g = gn;
          st_node = nn;
          st_pv = nn != NIL;
          st_hint = nn == NIL ? ohint : ((uint32_t)nn | (uint32_t)(dup || sc.cnt > 0) << 16);
        }
        STAMP_ADD(34, t_rp);
      }
    }
    STAMP_ADD(32, t_nl);
    STAMP_T t_e = STAMP_NOW();
    if (st_on) {
      c.nm_f[st_cell] = st_f;
      if (st_node != NIL) {
        if (st_pv) pvg_store(c, L, st_node, ci, st_g);
        open_cell(cells, st_cell, open_cgen, st_g, ci, c.gen2, st_hint);
      }
    }
    if (pend_on(pd)) {  // this pop's log entries, one store
      if (lane < pd.n) *(GAS v2u*)&((GAS uint32_t*)gp(c.A->open2))[2 * (pd.logn + lane)] = v2u{pd.lo, pd.hi};
      pd.logn += pd.n;
      pd.n = 0;
    }
    wave_lds_sync();
    STAMP_ADD(31, t_e);
  }
  *result = FLT_MAX;
  return true;
}

// AStar::find_path(int, int) (AStar.cpp:100-113); check_start = false: a_star_search from
// the soft-reset start node without the memo test of the start (AStar.cpp:88-95)
template <class CF>
__device__ __forceinline__ float holonomic(SearchCtx& c, AStarLdsT<CF>& L, int si, int sj, bool check_start = true) {
  const PlannerDev& P = *c.P;
  const SlotArena& A = *c.A;
  const int lane = c.lane;
  const size_t s_cell = (size_t)si * c.N + sj;
  STAMP_T t_hs = STAMP_NOW();
  if (check_start && ((c.visited[s_cell >> 5] >> (s_cell & 31)) & 1u)) return c.nm_f[s_cell];
  const float h0 = euclid_h(P, si, sj);
  c.nm_f[s_cell] = h0;  // Grid2D::set_start_node_grid -> Node2D::soft_reset
  c.asearch++;
  c.gen2++;
  c.ps2.next = 1;
  c.ps2.free = NIL;
  RBT<LdsAcc<CF>> tl;
  tl.s = lp(&L);
  tl.lane = lane;
  tl.cb = 0;
  tl.clear();
  L.kf[0].key = 0xffffffffu;
  Ring rg{0, 0};
  Pend pd{0u, 0u, 0, 0};  // the tree is deferred from the start
  {
    const SameCell none{0, NIL, 0.0f};
    const RankOut at0{0, NIL, 0.0f, NIL};
    int n0;
    insert_lds(c, tl, L, rg, ((uint32_t)si << 16) | (uint32_t)sj, h0, 0.0f, NIL, none, at0, &n0, pd);
    pvg_store(c, L, n0, NIL, 0.0f);  // {prev, g} of the start
    open_cell(c.cell2, (uint32_t)s_cell, c.gen2 - 1u, 0.0f, NIL, c.gen2, (uint32_t)n0);
  }
  wave_lds_sync();
  const int nact = P.diag ? 8 : 4;
  // this lane's action (Grid2D.cpp:22-40): nibble-packed (dx + 1, dy + 1) tables
  int adx = 0, ady = 0;
  float acost = 0.0f;
  if (lane < nact) {
    const uint32_t px = P.diag ? 0x00012221u : 0x0121u, py = P.diag ? 0x01222100u : 0x1210u;
    adx = (int)((px >> (4 * lane)) & 0xfu) - 1;
    ady = (int)((py >> (4 * lane)) & 0xfu) - 1;
    acost = (adx != 0 && ady != 0) ? P.act_cost_diag : P.act_cost_axis;
  }
  float result = FLT_MAX;
  STAMP_ADD(35, t_hs);
  if (HASTAR_LIKELY(astar_loop_lds(c, tl, L, rg, adx, ady, acost, &result, pd))) return result;
  if (pend_on(pd)) pend_replay(c, tl, L, pd);  // the migration copies the tree (into open2: the log is read first)
  // migrate the LDS tree to HBM nodes (identical indices) and continue there
  c.amigr++;
  GAS Node2* o2 = gp(A.open2);
  for (int base = 0; base < c.ps2.next; base += 64) {
    const int i = base + lane;
    // the colour shuffle runs with every lane active: a ds_bpermute reads 0 from a lane that
    // is off in EXEC, and lanes (i >> 5) of the last chunk can be (with a 2048-node pool the
    // colours of nodes 1984.. live in lanes 62, 63)
    const int col = (int)(((uint32_t)__shfl((int)tl.cb, i >> 5, 64) >> (i & 31)) & 1u);
    if (i < c.ps2.next) {
      Node2 n;
      const v2i pg = pvg_load(c, L, i);
      n.key = L.kf[i].key;
      n.f = L.kf[i].f;
      n.g = __int_as_float(pg.y);
      // a dead node's l is its free-list link, kept in f in LDS (free_lds)
      const bool dead = (uint32_t)n.key == 0xffffffffu && i > 0;  // (per lane: no uniform read)
      n.l = dead ? __float_as_int(L.kf[i].f) : L.lr[i].l;
      n.r = L.lr[i].r;
      n.p = L.p[i];
      n.color = col;
      n.prev = pg.x;
      gstore(&o2[i], n);
    }
  }
  wave_lds_sync();
  RBT<HbmAcc> th;
  th.t = o2;
  STAMP_T tg = STAMP_NOW();
  astar_loop<true>(c, th, adx, ady, acost, &result);
  STAMP_ADD(7, tg);
  return result;
}

// std::set<Node3D>::insert (HybridAStar.cpp:173, 191) into the outer open tree (HBM nodes
// behind the register cache, or the LDS tree of the latency kernel; the full 48-B record
// always goes to the arena's open3[n], the LDS tree keeps key/f/g/links of its nodes).
// where: optional {new node (NIL when the insert was dropped), parent, insert_left}
template <class OT>
__device__ __forceinline__ bool insert3(SearchCtx& c, OT& o3, const Succ& s, float f, int prev, int cap,
                                        int* where = nullptr) {
  bool left;
  const uint32_t key = key3(s.cx, s.cy, s.bin);
  STAMP_T tw = STAMP_NOW();
  const int pos = o3.insert_pos(key, f, &left);
  STAMP_ADD(19, tw);
  if (where) where[0] = NIL;
  if (HASTAR_UNLIKELY(pos == -2)) return true;
  const int n = tpool_alloc(o3, c.ps3, cap);
  if (HASTAR_UNLIKELY(n == NIL)) return false;
  if (where) {
    where[0] = n;
    where[1] = pos;
    where[2] = left ? 1 : 0;
  }
  Node3 d;
  d.key = key;
  d.f = f;
  d.l = NIL;
  d.r = NIL;
  d.p = pos;
  d.cc = (uint32_t)RB_RED | ((uint32_t)s.ci << 8);
  d.g = s.g;
  d.vmin = s.vmin;
  d.x = s.x;
  d.y = s.y;
  d.h = s.h;
  d.prev = prev;
  gstore(&c.open3[n], d);
  o3.fresh(n, d);
  STAMP_T tl = STAMP_NOW();
  o3.link(left, n, pos);
  STAMP_ADD(20, tl);
  return true;
}

// ---- the outer open tree in LDS (latency kernel) ------------------------------------------
// One search owns a CU: its outer open set (std::set<Node3D>, HybridAStar.h:72) keeps every
// node's tree part in LDS, 20 B per node: {key, f, l, r, p, colour} in one 16-B record (a walk
// step is one ds_read_b128) and g (the find-hit replacement test, HybridAStar.cpp:178).  The
// pose / vmin / prev payload stays in the arena's 48-B open3 record, read at the pop.  The
// open set of a cfg3 search peaks at a few hundred nodes (oracle census: 296 for query 0),
// of the batch's longest at 9,414; when the pool cannot take one more pop the tree moves to
// the HBM records (same indices: only links and colours are copied) and the search continues
// behind the register cache (RBT<CachedAcc3>).
constexpr int OUTER_LDS_CAP = 4688;  // (5504 before round 4: the helper waves' prep table took the rest)
struct alignas(16) Q3L {
  uint32_t key;
  float f;
  int16_t l, r, p;  // NIL = -1; indices < OUTER_LDS_CAP
  uint8_t col, pad;
};
static_assert(sizeof(Q3L) == 16, "one quad per outer LDS node");
struct OuterLds {
  Q3L q[OUTER_LDS_CAP];
  float g[OUTER_LDS_CAP];
};
// Path walks (as RBT<CachedAcc3>, rbtree_dev.h): lanes [0, plen) remember the last walk's
// nodes.  A new walk has every path lane read its node's current quad at once (one parallel
// ds_read_b128) and follows the path for as long as its own decision at depth d leads to the
// node at depth d + 1 under the current links: the shared prefix costs one LDS round trip and a
// ballot instead of a chain of dependent steps.  Links are re-read, never cached, so rotations,
// erases and reused indices need no bookkeeping: the prefix followed is the walk itself.
struct LdsAcc3 {
  static constexpr bool kPathWalk = true;
  LAS Q3L* q;
  LAS float* gg;
  GAS Node3* t;  // payload records (open3)
  int lane;
  int pid;       // this lane's node of the last walk's path (lane = depth)
  int plen;      // path lanes [0, plen) (wave-uniform)
  // the header's links (root, leftmost, rightmost) in wave-uniform registers as well, as
  // LdsAcc does: read without an LDS round trip, written to both (lds_tree loads them)
  int hp, hl, hr;
  __device__ __forceinline__ int L(int x) const { return x == 0 ? hl : ufi(q[x].l); }
  __device__ __forceinline__ int R(int x) const { return x == 0 ? hr : ufi(q[x].r); }
  __device__ __forceinline__ int P(int x) const { return x == 0 ? hp : ufi(q[x].p); }
  __device__ __forceinline__ int C(int x) const { return ufi(q[x].col); }
  __device__ __forceinline__ void sL(int x, int v) {
    q[x].l = (int16_t)v;
    hl = x == 0 ? v : hl;
  }
  __device__ __forceinline__ void sR(int x, int v) {
    q[x].r = (int16_t)v;
    hr = x == 0 ? v : hr;
  }
  __device__ __forceinline__ void sP(int x, int v) {
    q[x].p = (int16_t)v;
    hp = x == 0 ? v : hp;
  }
  __device__ __forceinline__ void sC(int x, int v) { q[x].col = (uint8_t)v; }
  __device__ __forceinline__ uint32_t K(int x) const { return ufu(q[x].key); }
  __device__ __forceinline__ float F(int x) const { return uff(q[x].f); }
  __device__ __forceinline__ float G(int x) const { return uff(gg[x]); }
  __device__ __forceinline__ Quad quad(int x) const {
    // one 16-B load (ds_read_b128) through memcpy: a byte-wise copy aliases every field
    // store, so it stays ordered after the 16-bit link stores (a vector-typed view of the
    // record would not, under type-based alias analysis)
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    v4u w;
    __builtin_memcpy(&w, (const Q3L*)&q[x], sizeof(Q3L));
    Quad o;
    o.key = ufu(w.x);
    o.f = uff(__uint_as_float(w.y));
    o.l = ufi((int)(int16_t)(w.z & 0xffffu));  // {l, r}: little-endian int16 pair
    o.r = ufi((int)(int16_t)(w.z >> 16));
    return o;
  }
  __device__ __forceinline__ Quad quad_at(int x, int depth) {
    if (lane == depth) pid = x;
    return quad(x);
  }
  // the walks of std::set::find / _M_get_insert_unique_pos: CachedAcc3::path_walk's contract
  __device__ __forceinline__ void path_walk(uint32_t k, float f, bool ins, int* y_, uint32_t* yk_, float* yf_,
                                            bool* comp_, int* rj_, uint32_t* rk_, float* rf_) {
    int y = 0, depth = 0;
    uint32_t yk = 0;
    float yf = 0.0f;
    bool comp = true;
    int rj = -1;
    uint32_t rk = 0;
    float rf = 0.0f;
    int x = P(0);
    if (x != NIL && plen > 0 && __builtin_amdgcn_readlane(pid, 0) == x) {
      const bool inpath = lane < plen;
      typedef uint32_t v4u __attribute__((ext_vector_type(4)));
      v4u w = {0u, 0u, 0xffffffffu, 0u};
      if (inpath) __builtin_memcpy(&w, (const Q3L*)&q[pid], sizeof(Q3L));
      const uint32_t ck = w.x;
      const float cf = __uint_as_float(w.y);
      const int cl = (int)(int16_t)(w.z & 0xffffu), cr = (int)(int16_t)(w.z >> 16);
      const bool left = ins ? rb_less(k, f, ck, cf) : !rb_less(ck, cf, k, f);
      const int child = left ? cl : cr;
      const int nxt = __shfl_down(pid, 1, 64);
      const bool cont = inpath && lane + 1 < plen && child == nxt;
      const uint64_t stop = __ballot(!cont);
      const int D = (int)__ffsll((unsigned long long)stop) - 1;  // node D is on the path; leave it via child
      const uint64_t below = D >= 63 ? ~0ull : ((2ull << D) - 1);
      const uint64_t lmask = __ballot(inpath && left) & below;
      if (ins) {
        y = __builtin_amdgcn_readlane(pid, D);
        yk = (uint32_t)__builtin_amdgcn_readlane((int)ck, D);
        yf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), D));
        comp = (lmask >> D) & 1ull;
        const uint64_t rmask = __ballot(inpath && !left) & below;
        if (rmask) {
          const int h = 63 - __builtin_clzll(rmask);
          rj = __builtin_amdgcn_readlane(pid, h);
          rk = (uint32_t)__builtin_amdgcn_readlane((int)ck, h);
          rf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), h));
        }
      } else if (lmask) {
        const int h = 63 - __builtin_clzll(lmask);
        y = __builtin_amdgcn_readlane(pid, h);
        yk = (uint32_t)__builtin_amdgcn_readlane((int)ck, h);
        yf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), h));
      }
      x = __builtin_amdgcn_readlane(child, D);
      depth = D + 1;
    }
    while (x != NIL) {
      const Quad qq = quad_at(x, depth++);
      if (ins) {
        y = x;
        yk = qq.key;
        yf = qq.f;
        comp = rb_less(k, f, qq.key, qq.f);
        if (!comp) {
          rj = y;
          rk = yk;
          rf = yf;
        }
        x = comp ? qq.l : qq.r;
      } else if (!rb_less(qq.key, qq.f, k, f)) {
        y = x;
        yk = qq.key;
        yf = qq.f;
        x = qq.l;
      } else {
        x = qq.r;
      }
    }
    plen = depth < 64 ? depth : 64;
    *y_ = y;
    *yk_ = yk;
    *yf_ = yf;
    *comp_ = comp;
    *rj_ = rj;
    *rk_ = rk;
    *rf_ = rf;
  }
  __device__ __forceinline__ void leaf(int x, int p) {
    q[x].l = (int16_t)NIL;
    q[x].r = (int16_t)NIL;
    q[x].p = (int16_t)p;
    q[x].col = (uint8_t)RB_RED;
  }
  // a node just written to open3[x] by insert3: its tree part (links come with link())
  __device__ __forceinline__ void fresh(int x, const Node3& n) {
    q[x].key = n.key;
    q[x].f = n.f;
    gg[x] = n.g;
  }
  __device__ __forceinline__ void reset_cache() { plen = 0; }
  // the popped node: key/f/links from LDS, the payload from its HBM record
  __device__ __forceinline__ Node3 node(int x) const { return node_q(x, quad(x)); }
  // the same with its quad already read (the pop issues its closed-set probe in between)
  __device__ __forceinline__ Node3 node_q(int x, const Quad& a) const {
    typedef int v4 __attribute__((ext_vector_type(4)));
    const GAS v4* h = (const GAS v4*)&t[x];
    return node_pv(a, h[1], h[2]);
  }
  // ... and with its payload quads already loaded (PopPrefetch)
  template <class V4>
  __device__ __forceinline__ Node3 node_pv(const Quad& a, const V4& b, const V4& d) const {
    Node3 n;
    n.key = a.key;
    n.f = a.f;
    n.l = a.l;
    n.r = a.r;
    n.p = ufi(b.x);
    n.cc = ufu((uint32_t)b.y);
    n.g = uff(__int_as_float(b.z));
    n.vmin = uff(__int_as_float(b.w));
    n.x = uff(__int_as_float(d.x));
    n.y = uff(__int_as_float(d.y));
    n.h = uff(__int_as_float(d.z));
    n.prev = ufi(d.w);
    return n;
  }
};
__device__ __forceinline__ RBT<LdsAcc3> lds_tree(OuterLds& ol, const SearchCtx& c) {
  RBT<LdsAcc3> t;
  t.q = lp(ol.q);
  t.gg = lp(ol.g);
  t.t = c.open3;
  t.lane = c.lane;
  t.pid = NIL;
  t.plen = 0;
  t.hp = ufi(t.q[0].p);
  t.hl = ufi(t.q[0].l);
  t.hr = ufi(t.q[0].r);
  return t;
}
// LDS tree -> HBM records (links and colours; key, f, g and the payload are there already),
// for every pool index in use, the header (0) and free-list nodes included
__device__ __forceinline__ void lds_outer_store(SearchCtx& c, OuterLds& ol, int lane) {
  GAS Node3* t = c.open3;
  const LAS Q3L* q = lp(ol.q);
  for (int i = lane; i < c.ps3.next; i += 64) {
    t[i].l = q[i].l;
    t[i].r = q[i].r;
    t[i].p = q[i].p;
    *(GAS uint8_t*)&t[i].cc = q[i].col;  // byte 0 only: the curvature index stays
  }
  wave_lds_sync();
}
// HBM records -> LDS tree (a resumed search whose pool fits); false when it does not fit
__device__ __forceinline__ bool lds_outer_load(SearchCtx& c, OuterLds& ol, int lane) {
  if (c.ps3.next > OUTER_LDS_CAP - 64) return false;
  const GAS Node3* t = c.open3;
  LAS Q3L* q = lp(ol.q);
  LAS float* g = lp(ol.g);
  for (int i = lane; i < c.ps3.next; i += 64) {
    const Node3 n = gload(&t[i]);
    q[i].key = n.key;
    q[i].f = n.f;
    q[i].l = (int16_t)n.l;
    q[i].r = (int16_t)n.r;
    q[i].p = (int16_t)n.p;
    q[i].col = (uint8_t)(n.cc & 0xffu);
    q[i].pad = 0;
    g[i] = n.g;
  }
  wave_lds_sync();
  return true;
}


// ---- expansion prep: helper waves of the latency kernel ------------------------------------
// The latency kernel runs one search per CU with one wavefront, so three SIMDs of its CU idle.
// Its workgroup has three more waves that PRE-compute expansions: a node's successors
// (VehicleModel.cpp:63-105: poses, speed limits, bins, cells, the occupancy filter of
// Grid3D.cpp:54-59), their APF fields (Grid3D.cpp:206-227) and Dubins lengths (Dubins.cpp:19-69)
// are pure functions of the node's pose, speed, curvature index and the search's map, not of the
// search state.  The main wave posts every successor it may insert; a helper computes that
// successor's own expansion while the main wave goes on (finds, inner A*, inserts); when the main
// wave later pops a node whose inputs match a finished entry bit for bit, it takes the entry
// instead of computing it.  Entries are tagged with the search's epoch and hold their inputs, so a
// result can only be used for exactly the inputs it was computed from: results are identical
// by construction (tests/test_gpu_*: every latency-kernel case).
//
// A ring of PREP_E entries in LDS (request seq s lives in entry s % PREP_E); state word per entry:
// seq << 2 | phase, phase 0 = empty / being written by the main wave, 1 = posted, 2 = a helper
// computes it, 3 = done.  The main wave overwrites only entries that no helper holds (a CAS to
// phase 0); a helper claims a posted entry by CAS 1 -> 2 and alone moves it 2 -> 3.
constexpr int PREP_E = 64;   // entries, one per lane (the latest requests: with 32, 77 % of cfg5's warm pops found theirs)
constexpr int PREP_C = 4;    // candidates per entry: action windows of at most 4 (16-lane groups)
constexpr int PREP_HELPERS = 3;
struct alignas(16) PrepIn {  // the inputs of one expansion
  uint32_t key;
  float x, y, h, vmin;
  int ci;
  uint32_t epoch, pad;
};
struct alignas(16) PrepCand {  // one candidate successor of that expansion
  float sx, sy, sh, vm, fc, dub, oact;
  uint32_t skey;
  uint32_t flags;  // bit 0: feasible (speed limit), bit 1: cell in the grid, bit 2: kept (bit 1 and occ < thr)
  uint32_t pad0, pad1, pad2;
};
struct PrepShared {
  PrepIn in[PREP_E];
  PrepCand out[PREP_E][PREP_C];
  uint32_t state[PREP_E];
  uint32_t tail;                    // requests posted so far (main wave)
  uint32_t epoch;                   // the current search (main wave)
  uint32_t stop;                    // the kernel is done (main wave)
  uint32_t pad;
  int pidx;                         // the planner of `epoch` (its index in the kernel's descriptors)
  int pad1;
  ApfCand kept[PREP_HELPERS][APF_MAXC];  // the helpers' APF cull buffers
};

typedef LAS PrepShared PrepL;
__device__ __forceinline__ uint32_t prep_ld(LAS uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void prep_st(LAS uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool prep_cas(LAS uint32_t* p, uint32_t expect, uint32_t v) {
  return __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
}

// main wave: the entry holding the expansion of `cur` (a closed record: the popped node, or the
// old record of its key), waiting for a helper still computing it; -1 if there is none
__device__ __forceinline__ int prep_find(PrepL& pr, uint32_t key, float x, float y, float h, float vmin, int ci,
                                         uint32_t epoch, int lane) {
  const int e = lane & (PREP_E - 1);
  const uint32_t st = prep_ld(&pr.state[e]);
  PrepIn in;
  __builtin_memcpy(&in, (const PrepIn*)&pr.in[e], sizeof(in));
  const bool match = lane < PREP_E && (st & 3u) >= 2u && in.epoch == epoch && in.key == key &&
                     __float_as_uint(in.x) == __float_as_uint(x) && __float_as_uint(in.y) == __float_as_uint(y) &&
                     __float_as_uint(in.h) == __float_as_uint(h) && __float_as_uint(in.vmin) == __float_as_uint(vmin) &&
                     in.ci == ci;
  const uint64_t m = __ballot(match);
  if (!m) return -1;
  const int e0 = (int)__ffsll((unsigned long long)m) - 1;
  uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane((int)st, e0);
  // a helper holds it: it finishes this one expansion (about the main wave's own cost of it)
  while ((s0 & 3u) == 2u) {
    __builtin_amdgcn_s_sleep(1);
    s0 = ufu(prep_ld(&pr.state[e0]));
  }
  return (s0 & 3u) == 3u ? e0 : -1;
}

// main wave: post the kept successors of this expansion (candidate a of the window in lanes
// [16 a, 16 a + 16), lead lane 16 a), newest last
__device__ __forceinline__ void prep_post(PrepL& pr, bool post, uint32_t skey, float sx, float sy, float sh,
                                          float vm, int ci, uint32_t epoch, int lane) {
  const uint64_t m = __ballot(post);
  if (!m) return;
  const uint32_t tail = ufu(pr.tail);
  if (post) {
    const uint32_t k = (uint32_t)__popcll(m & ((1ull << lane) - 1));
    const uint32_t seq = tail + k + 1u;  // >= 1
    const int e = (int)(seq & (PREP_E - 1));
    const uint32_t old = prep_ld(&pr.state[e]);
    if ((old & 3u) != 2u && prep_cas(&pr.state[e], old, seq << 2)) {
      PrepIn in;
      in.key = skey;
      in.x = sx;
      in.y = sy;
      in.h = sh;
      in.vmin = vm;
      in.ci = ci;
      in.epoch = epoch;
      in.pad = 0;
      __builtin_memcpy((PrepIn*)&pr.in[e], &in, sizeof(in));
      prep_st(&pr.state[e], (seq << 2) | 1u);
    }
  }
  if (lane == 0) pr.tail = tail + (uint32_t)__popcll(m);
  wave_lds_sync();
}

// helper wave h (1..3): claim the newest posted expansion, compute it, publish it; returns when
// the main wave has set `stop`
__device__ void prep_helper(PrepL& pr, ApfStage& apfs, const PlannerDev* __restrict__ descs, int h, int lane) {
  ApfCand* kept_buf = (ApfCand*)pr.kept[h - 1];
  for (;;) {
    const int e = lane & (PREP_E - 1);
    const uint32_t st = prep_ld(&pr.state[e]);
    const bool posted = lane < PREP_E && (st & 3u) == 1u;
    // the newest posted request (largest seq)
    uint32_t best = posted ? (st >> 2) : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) best = max(best, (uint32_t)__shfl_xor((int)best, o, 64));
    best = ufu(best);
    if (best == 0u) {
      if (ufu(prep_ld(&pr.stop))) return;
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    const int be = (int)(best & (PREP_E - 1));
    bool won = false;
    if (lane == 0) won = prep_cas(&pr.state[be], (best << 2) | 1u, (best << 2) | 2u);
    if (!__builtin_amdgcn_readfirstlane((int)won)) continue;
    PrepIn in;
    __builtin_memcpy(&in, (const PrepIn*)&pr.in[be], sizeof(in));
    const PlannerDev* Pp = descs + ufi(pr.pidx);
    const uint32_t epoch = ufu(prep_ld(&pr.epoch));
    if (ufu(in.epoch) == epoch) {
      const PlannerDev& P = *Pp;
      const uint32_t key = ufu(in.key);
      const float cx = uff(in.x), cy = uff(in.y), ch = uff(in.h), cvm = uff(in.vmin);
      const int cci = ufi(in.ci), cbin = key3_bin(key);
      const bool slow = cvm < 1.0f;
      int lo = cci - P.na;
      lo = lo < 0 ? 0 : lo;
      const int span = 2 * P.na + 1;
      const int ca = lane >> 4, sub = lane & 15;
      const int ai = lo + ca;
      bool cand = ca < span && ai < P.nsteer;
      const int ia = cand ? ai : lo;
      const float cabs = gp(P.curv_abs)[ia];
      const GAS float* ofs = &gp(P.off)[2 * ((size_t)ia * (P.bins + 1) + cbin)];
      const float ofx = ofs[0], ofy = ofs[1], odth = gp(P.dth)[ia], oact = gp(P.act_cost)[ia];
      float vm = 0.0f;
      if (cand && !slow) {
        const float lat = cvm * cabs;
        if (lat > P.a_lat) cand = false;
        const float al = (float)sqrt(1.0 - (double)((lat * lat) / P.a_lat2));
        vm = cvm - 2.0f * al * P.ts;
      }
      float sx = 0.0f, sy = 0.0f, sh = 0.0f;
      int sbin = 0, scx = 0, scy = 0;
      bool inb = false;
      if (cand) {
        sx = cx + ofx;
        sy = cy + ofy;
        sh = wrap_pi_f(ch + odth);
        sbin = heading_bin(sh, P.prec);
        scx = trunc_f(sx / P.res);
        scy = trunc_f(sy / P.res);
        inb = scx > -1 && scx < P.N && scy > -1 && scy < P.N;
      }
      const bool lead = inb && sub == 0;
      float occv = 0.0f;
      if (lead) occv = gp(P.occ)[(size_t)scx * P.N + scy];
      const GoalC GC = goal_centres(P.r_min, P.goal_x, P.goal_y, P.goal_h);
      const float dub = cand_dubins(P.r_min, GC, P.goal_h, sx, sy, sh, 16, lane);
      const float fc = apf_fused_k(P, apfs, kept_buf, cx, cy, sx, sy, sh, __ballot(lead), 16, lane);
      const bool kept = lead && occv < P.thr;
      if (sub == 0 && ca < PREP_C) {
        PrepCand o;
        o.sx = sx;
        o.sy = sy;
        o.sh = sh;
        o.vm = vm;
        o.fc = fc;
        o.dub = dub;
        o.oact = oact;
        o.skey = key3(scx, scy, sbin);
        o.flags = (cand ? 1u : 0u) | (inb ? 2u : 0u) | (kept ? 4u : 0u);
        o.pad0 = o.pad1 = o.pad2 = 0u;
        __builtin_memcpy((PrepCand*)&pr.out[be][ca], &o, sizeof(o));
      }
    }
    wave_lds_sync();
    if (lane == 0) prep_st(&pr.state[be], (best << 2) | 3u);
  }
}

// The loop of hybrid_a_star_search (HybridAStar.cpp:107-194) over outer open tree OT: the
// HBM tree behind the register cache (RBT<CachedAcc3>) or the latency kernel's LDS tree
// (RBT<LdsAcc3>).  Returns LOOP_DONE (the search ended: goal, shot, empty open set or a
// status), LOOP_PARKED (the arena cannot take one more pop) or LOOP_MIGRATE (LDS tree only:
// its pool or the closed records are about to fill; the caller moves the tree to HBM and
// continues there, at the same pop).
constexpr int LOOP_DONE = 0, LOOP_PARKED = 1, LOOP_MIGRATE = 2, LOOP_HANDOFF = 3;

// ---- handoff of a long batch-kernel search to a free latency CU (HandoffBoard, hastar_layout.h)
// Every board word another CU polls is accessed by agent-scope atomics (write-through, no stale
// L1 copy); the search state itself (arena records, SearchResult, the planner's maps) is
// published by the batch wave's agent-scope release before READY and read by the latency wave
// after its agent-scope acquire (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ uint32_t ho_ld(GAS uint32_t* p) {
  return __hip_atomic_load((uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ho_st(GAS uint32_t* p, uint32_t v) {
  __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ho_ld64(GAS uint64_t* p) {
  const uint32_t lo = ho_ld((GAS uint32_t*)p), hi = ho_ld((GAS uint32_t*)p + 1);
  return ((uint64_t)hi << 32) | lo;
}
// the board of a split launch's batch-kernel wave, or null (no split launch, an arena without
// a board, or an arena index past the board)
__device__ __forceinline__ GAS HandoffBoard* ho_board(const SearchCtx& c) {
  GAS HandoffBoard* hb = gp(c.A->board);
  if (hb == nullptr || c.slot >= HANDOFF_CAP || hb->enabled == 0) return nullptr;
  return hb;
}
// Batch kernel, at a pop boundary every 64 pops: offer the search once it has run thr pops;
// true when a latency wave has claimed the offer (the caller parks the search for it).
__device__ __forceinline__ bool ho_poll(SearchCtx& c) {
  GAS HandoffBoard* hb = ho_board(c);
  if (hb == nullptr || c.pops < (uint32_t)hb->thr) return false;
  GAS uint32_t* st = &hb->state[c.slot];
  const uint32_t v = (uint32_t)__builtin_amdgcn_readfirstlane((int)ho_ld(st));
  if (v == HANDOFF_CLAIMED) return true;
#ifndef BISECT_NOPOST
  if (v == HANDOFF_EMPTY && c.lane == 0) {
    GAS HandoffEntry* e = &hb->entry[c.slot];
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    ho_st((GAS uint32_t*)&e->t_start, (uint32_t)t);
    ho_st((GAS uint32_t*)&e->t_start + 1, (uint32_t)(t >> 32));
    ho_st((GAS uint32_t*)&e->slot, (uint32_t)c.slot);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the entry before its state
    ho_st(st, HANDOFF_POSTED);
    atomicAdd((int*)&hb->posted, 1);
  }
#endif
  return false;
}
// Batch kernel, after a search that may have offered itself (not handed over): withdraw the
// offer, or release a claimer that came too late.
__device__ __forceinline__ void ho_withdraw(SearchCtx& c) {
  GAS HandoffBoard* hb = ho_board(c);
  if (hb == nullptr || c.pops < (uint32_t)hb->thr) return;
  if (c.lane == 0) {
    GAS uint32_t* st = &hb->state[c.slot];
    const uint32_t old = atomicCAS((uint32_t*)st, HANDOFF_POSTED, HANDOFF_EMPTY);
    if (old == HANDOFF_POSTED) atomicSub((int*)&hb->posted, 1);
    else if (old == HANDOFF_CLAIMED) ho_st(st, HANDOFF_CANCELLED);
  }
}
// Latency kernel, LDS tree: right after a pop, the HBM reads of the NEXT pop (the payload of the
// tree's new leftmost node and its closed-set probe) are issued, so they arrive during the
// expansion.  The next pop takes them when its node is that one (no successor went before it,
// and the node was not freed in between); the closed set only changes at pops, so the probe
// is still current.
struct PopPrefetch {
  typedef int v4 __attribute__((ext_vector_type(4)));
  int idx;     // node index, NIL = none
  uint32_t ph; // its closed-set hash slot
  v2u probe;   // the slot's {key, gen | idx}
  v4 b, d;     // payload quads 1 and 2 of open3[idx]
};
struct LoopState {
  int counter, interval;
  bool shot_allowed;
  uint64_t dig;
  int ok, via_shot, terminal, dub_n;
  float cost;
};
template <class CF, bool kLdsOuter, bool kPrep, class OT>
__device__ __forceinline__ int search_loop(SearchCtx& c, OT& o3, ApfStage& apfs, AStarLdsT<CF>& alds, LoopState& S,
                                           long long hard_pops, int closed_lim, int open_lim, int open_cap,
                                           PrepL* pr = nullptr) {
  const PlannerDev& P = *c.P;
  const SlotArena& A = *c.A;
  const int lane = c.lane;
  int& counter = S.counter;
  int& interval = S.interval;
  bool& shot_allowed = S.shot_allowed;
  uint64_t& dig = S.dig;
  int& ok = S.ok;
  int& via_shot = S.via_shot;
  int& terminal = S.terminal;
  int& dub_n = S.dub_n;
  float& cost = S.cost;
  bool parked = false;
  const float r = P.r_min;
  const GoalC GC = goal_centres(r, P.goal_x, P.goal_y, P.goal_h);
  const int span = 2 * P.na + 1;
  const int open_lim_t = kLdsOuter ? min(open_lim, open_cap) : open_lim;
  PopPrefetch pf;  // issued after the pop
  pf.idx = NIL;
  pf.ph = 0u;
  pf.probe = v2u{0u, 0u};
  pf.b = PopPrefetch::v4{0, 0, 0, 0};
  pf.d = pf.b;
  // lanes per candidate action: 16 when the window has at most 4 actions (the Dubins
  // libm calls then spread over the group), else 4 (one Dubins word per lane)
#ifdef HASTAR_DBG_NARROW
  const int gsh = 2, gs = 4;
#else
  const int gsh = span <= 4 ? 4 : 2, gs = 1 << gsh;
#endif
  while (!o3.empty()) {
    if (HASTAR_UNLIKELY(hard_pops > 0 && c.pops >= hard_pops)) { c.status = -75; break; }
    // one more pop needs a closed record and at most `span` open nodes (the pop frees one)
    if (HASTAR_UNLIKELY(c.n_closed3 + 1 >= closed_lim || c.ps3.next + span + 1 > open_lim_t)) {
      if (kLdsOuter) return LOOP_MIGRATE;  // the HBM loop continues (and parks if it must)
      parked = true;
      break;
    }
    if constexpr (!kPrep) {  // batch kernel: a free latency CU may take this search over
#ifndef BISECT_NOPOLL
      if (HASTAR_UNLIKELY((c.pops & 63u) == 0u) && HASTAR_UNLIKELY(ho_poll(c))) return LOOP_HANDOFF;
#endif
    }
    STAMP_T tp = STAMP_NOW();
    const int b = o3.begin();
    // the closed-set probe is issued first; its HBM latency overlaps the erase, which
    // does not depend on it (HybridAStar.cpp:109-111 order is kept: the insert itself
    // reads the popped node's fields, captured in `top`).  HBM tree: the node is usually
    // cached (the leftmost node was touched by the last walks).  LDS tree: the key comes from
    // LDS, so the probe and the payload's HBM read are in flight together.
    uint32_t ph;
    v2u p0;
    Node3 top;
    if constexpr (kLdsOuter) {
      const Quad tq = o3.quad(b);
      if (b == pf.idx) {
        ph = pf.ph;
        p0 = pf.probe;
        top = o3.node_pv(tq, pf.b, pf.d);
      } else {
        p0 = closed3_probe(c, tq.key, &ph);
        top = o3.node_q(b, tq);
      }
#ifdef HASTAR_STAMPS
      if (b == pf.idx) c.cyc[38]++;  // pops served by a prefetch
      else c.cyc[39]++;
#endif
    } else {
      top = o3.node(b);
      p0 = closed3_probe(c, top.key, &ph);
    }
    o3.unlink(b);
    tpool_free(o3, c.ps3, b);
    bool fresh;
    const int ci = closed3_insert(c, top, &fresh, ph, p0);
    if (HASTAR_UNLIKELY(ci == NIL)) { c.status = -75; break; }
    // a duplicate key expands the OLD record; a new record is the popped node itself
    Closed3 cur;
    if (fresh) {
      cur.key = top.key;
      cur.g = top.g;
      cur.vmin = top.vmin;
      cur.prev = top.prev;
      cur.x = top.x;
      cur.y = top.y;
      cur.h = top.h;
      cur.ci = (int)(top.cc >> 8);
    } else {
      cur = gload(&c.closed3[ci]);
    }
    c.pops++;
    const int cx = key3_x(cur.key), cy = key3_y(cur.key), cbin = key3_bin(cur.key);
    dig = mix64(dig ^ digest_key(cur.key)) + (uint64_t)fbits(cur.g);
    if constexpr (kLdsOuter) {
      const int b2 = o3.begin();
      pf.idx = NIL;
      if (b2 != 0) {
        typedef int v4 __attribute__((ext_vector_type(4)));
        pf.probe = closed3_probe(c, o3.K(b2), &pf.ph);
        const GAS v4* h2 = (const GAS v4*)&c.open3[b2];
        pf.b = h2[1];
        pf.d = h2[2];
        pf.idx = b2;
      }
    }
    STAMP_ADD(0, tp);
    // goal test: Node3D::operator== compares the cell only (Node3D.h:42)
    if (HASTAR_UNLIKELY(cx == P.goal_cx && cy == P.goal_cy)) {
      terminal = ci;
      cost = cur.g;
      ok = 1;
      break;
    }
    if (shot_allowed) {
      if (HASTAR_UNLIKELY(++counter == interval)) {
        STAMP_T tsh = STAMP_NOW();
        c.shots++;
        int word = 0;
        float prm[4];
        // Dubins::get_shortest_path (Dubins.cpp:125-153)
        const float L = dubins_shortest(r, cur.x, cur.y, cur.h, P.goal_x, P.goal_y, P.goal_h, &word, prm);
        const Centres C = dubins_centres(r, cur.x, cur.y, cur.h, P.goal_x, P.goal_y, P.goal_h);
        // the shot counts only when its first arc turns <= 90 degrees (Dubins.cpp:125-153); the
        // samples are checked as they are made (Grid3D::check_path), so a blocked shot stops at
        // its first blocked chunk
        const bool first_arc_long = fabsf(prm[1]) > (float)M_PI_2;
        const int n = first_arc_long
                          ? dubins_sample<2>(P, C, word, prm, gp(A.dub_xyh), gp(A.dub_curv), A.dub_cap, lane)
                          : dubins_sample<1>(P, C, word, prm, gp(A.dub_xyh), gp(A.dub_curv), A.dub_cap, lane);
        if (HASTAR_UNLIKELY(n == -1)) { c.status = -75; break; }
        wave_lds_sync();
        if (HASTAR_UNLIKELY(!first_arc_long && n > 0)) {
          terminal = cur.prev;
          cost = cur.g + L;
          ok = 1;
          via_shot = 1;
          dub_n = n;
          break;
        }
        counter = 0;
        interval = max(interval - P.shot_decay, 50);
        STAMP_ADD(4, tsh);
      }
    }
    // ---- successors (VehicleModel::get_neighbors, VehicleModel.cpp:63-105; Grid3D filter and
    // field, Grid3D.cpp:47-74, 206-227) and their Dubins lengths (Dubins.cpp:19-69), fused.
    // Candidate a of the action window [lo, lo + span) is evaluated by lanes
    // [a * gs, (a + 1) * gs).  The HBM probes of every candidate (occupancy, closed-set slot,
    // memo flag and value) are issued first, so their latency hides behind the Dubins and
    // APF arithmetic; the kept successors keep the reference's push_back (action) order.
    STAMP_T tx = STAMP_NOW();
    shot_allowed = cur.vmin < 1.0f;
    int lo = cur.ci - P.na;
    lo = lo < 0 ? 0 : lo;
    const int ca = lane >> gsh, sub = lane & (gs - 1);
    const int ai = lo + ca;
    bool cand = ca < span && ai < P.nsteer;
    const int ia = cand ? ai : lo;  // in-range index: the table loads are unconditional
    // latency kernel: a helper wave may have computed this expansion already (bit for bit the
    // values below: the same code on the same inputs, prep_helper)
    int pe = -1;
    if constexpr (kPrep) {
      if (gs == 16 && pr) pe = prep_find(*pr, cur.key, cur.x, cur.y, cur.h, cur.vmin, cur.ci, c.prep_epoch, lane);
#ifdef HASTAR_STAMPS
      if (gs == 16 && pr && pe >= 0) c.cyc[36]++;  // prepared expansions taken
      if (gs == 16 && pr && pe < 0) c.cyc[37]++;   // computed here
#endif
    }
    float vm = 0.0f, sx = 0.0f, sy = 0.0f, sh = 0.0f, sg = 0.0f, dub = 0.0f, fc = 0.0f;
    int sbin = 0, scx = 0, scy = 0;
    bool inb = false, pkept = false;
    if (kPrep && pe >= 0) {
      PrepCand pc;
      __builtin_memcpy(&pc, (const PrepCand*)&pr->out[pe][ca & (PREP_C - 1)], sizeof(pc));
      cand = cand && ca < PREP_C && (pc.flags & 1u);
      if (cand) {
        sx = pc.sx;
        sy = pc.sy;
        sh = pc.sh;
        vm = pc.vm;
        sg = cur.g + pc.oact;
        sbin = key3_bin(pc.skey);
        scx = key3_x(pc.skey);
        scy = key3_y(pc.skey);
        inb = (pc.flags & 2u) != 0u;
        pkept = (pc.flags & 4u) != 0u;
        dub = pc.dub;
        fc = pc.fc;
      }
    } else {
      const float cabs = gp(P.curv_abs)[ia];
      const GAS float* ofs = &gp(P.off)[2 * ((size_t)ia * (P.bins + 1) + cbin)];
      const float ofx = ofs[0], ofy = ofs[1], odth = gp(P.dth)[ia], oact = gp(P.act_cost)[ia];
      if (cand && !shot_allowed) {
        const float lat = cur.vmin * cabs;
        if (lat > P.a_lat) cand = false;
        const float al = (float)sqrt(1.0 - (double)((lat * lat) / P.a_lat2));
        vm = cur.vmin - 2.0f * al * P.ts;
      }
      if (cand) {
        sx = cur.x + ofx;
        sy = cur.y + ofy;
        sh = wrap_pi_f(cur.h + odth);
        sg = cur.g + oact;
        sbin = heading_bin(sh, P.prec);
        scx = trunc_f(sx / P.res);
        scy = trunc_f(sy / P.res);
        inb = scx > -1 && scx < c.N && scy > -1 && scy < c.N;
      }
    }
    const bool lead = inb && sub == 0;
    const uint32_t skey = key3(scx, scy, sbin);
    uint32_t sh0 = 0;
    v2u slot0{0u, 0u};
    float occv = 0.0f, pnf = 0.0f;
    uint32_t pvis = 0;
    if (lead) {
      const size_t cell = (size_t)scx * c.N + scy;
      if (!kPrep || pe < 0) occv = c.occ[cell];
      sh0 = slot_hash(skey) & c.smask;
      slot0 = *(const GAS v2u*)&c.slots3[sh0];
      pvis = (c.visited[cell >> 5] >> (cell & 31)) & 1u;
      pnf = c.nm_f[cell];
    }
    STAMP_ADD(16, tx);
    if (!kPrep || pe < 0) {
      STAMP_T tdub = STAMP_NOW();
      dub = cand_dubins(r, GC, P.goal_h, sx, sy, sh, gs, lane);
      STAMP_ADD(18, tdub);
      STAMP_T tapf = STAMP_NOW();
      fc = apf_fused(P, apfs, cur.x, cur.y, sx, sy, sh, __ballot(lead), gs, lane);
      STAMP_ADD(17, tapf);
    }
    STAMP_T tw = STAMP_NOW();
    const bool kept = lead && ((kPrep && pe >= 0) ? pkept : occv < c.thr);
    // hand the kept successors to the helper waves: the next pops are mostly among them
    if constexpr (kPrep) {
      if (gs == 16 && pr) prep_post(*pr, kept, skey, sx, sy, sh, vm, lo + ca, c.prep_epoch, lane);
    }
    const uint64_t km = __ballot(kept);
    c.succ += __popcll(km);
    // closed-set membership (continuing each kept candidate's probe sequence; the closed
    // set does not change while the successors are processed)
    bool isc = false;
    if (kept) {
      const uint32_t gbits = (c.gen3 & SLOT3_GEN_MASK) << SLOT3_IDX_BITS;
      uint32_t hs = sh0;
      v2u sv = slot0;
      for (;;) {
        if ((sv.y & ~SLOT3_IDX_MASK) != gbits) break;
        if (sv.x == skey) {
          isc = true;
          break;
        }
        hs = (hs + 1) & c.smask;
        sv = *(const GAS v2u*)&c.slots3[hs];
      }
    }
    const uint64_t closed_m = __ballot(isc);
    const uint64_t vis_m = __ballot(kept && pvis != 0u);
    STAMP_ADD(21, tw);
    STAMP_ADD(1, tx);
    // ---- HybridAStar.cpp:159-193, successors in action order
    STAMP_T tb = STAMP_NOW();
    bool fail = false;
#ifdef HASTAR_DBG_NOPREF
    bool memo_ok = false;
#else
    bool memo_ok = true;  // no inner A* search has run since the memo probes were issued
#endif
    for (uint64_t m = km & ~closed_m; m; m &= m - 1) {
      const int L = __ffsll((unsigned long long)m) - 1;
      Succ s;
      s.x = rl_f(sx, L);
      s.y = rl_f(sy, L);
      s.h = rl_f(sh, L);
      s.g = rl_f(sg, L) + rl_f(fc, L);  // Grid3D.cpp:66-69: g += field
      s.vmin = rl_f(vm, L);
      s.ci = lo + (L >> gsh);
      s.bin = rl_i(sbin, L);
      s.cx = rl_i(scx, L);
      s.cy = rl_i(scy, L);
      s.dub = rl_f(dub, L);
      const uint32_t key = key3(s.cx, s.cy, s.bin);
      STAMP_T tf3 = STAMP_NOW();
      // std::set::find with f == g (the heuristic is not added yet).  The tree's in-order
      // f sequence is strictly increasing, so when g <= f(leftmost) the lower_bound
      // predicate (key != k && f < g) is false at every node: the walk ends at the
      // leftmost node whatever the shape, and it matches iff its key is k or f == g.
      int hit;
      {
        const int lm = o3.begin();
        const float lf = lm != 0 ? o3.F(lm) : 0.0f;
        if (lm == 0) hit = 0;
        else if (s.g <= lf) hit = (o3.K(lm) == key || s.g >= lf) ? lm : 0;
        else hit = o3.find(key, s.g);
      }
      STAMP_ADD(13, tf3);
      const bool repl = hit != 0 && s.g < o3.G(hit);
      if (HASTAR_LIKELY(hit == 0 || repl)) {
        if (HASTAR_UNLIKELY(repl)) {
          STAMP_T tu3 = STAMP_NOW();
          o3.unlink(hit);
          tpool_free(o3, c.ps3, hit);
          if (kLdsOuter && hit == pf.idx) pf.idx = NIL;  // its index may be reused by the insert
          STAMP_ADD(15, tu3);
        }
        // AStar::find_path(int, int): a memo hit probed above is still valid while no
        // A* search has run in this expansion (only a search writes the memo)
        STAMP_T ta = STAMP_NOW();
        float h1;
        if (memo_ok && ((vis_m >> L) & 1ull)) {
          h1 = rl_f(pnf, L);
        } else {
          const long long a0 = c.asearch;
          h1 = holonomic(c, alds, s.cx, s.cy);
          if (c.asearch != a0) memo_ok = false;
        }
        STAMP_ADD(3, ta);
        const float f = s.g + stl_max(h1, s.dub);
        STAMP_T ti3 = STAMP_NOW();
        if (HASTAR_UNLIKELY(!insert3(c, o3, s, f, ci, open_cap))) { fail = true; break; }
        STAMP_ADD(14, ti3);
      }
      if (HASTAR_UNLIKELY(c.status != 0)) break;
    }
    wave_lds_sync();
    STAMP_ADD(2, tb);
    if (HASTAR_UNLIKELY(fail)) c.status = -75;
    if (HASTAR_UNLIKELY(c.status != 0)) break;
  }
  return parked ? LOOP_PARKED : LOOP_DONE;
}

// ------------------------------------------------------------------- the search -------
// One find_path (HybridAStar.cpp:68-88 incl. hybrid_a_star_search 93-199 and
// reconstruct_path 208-262) of planner *c.P in arena *c.A, run by one wavefront.
// Returns true when the search parked (its arena could not take one more pop; the state
// stays in this arena, see SearchResult).  resume: continue a parked search whose records
// the host copied into this (larger) arena.  hard_pops > 0 ends a search after that many
// pops with HASTAR_EOVERFLOW (an explicit budget; 0 = none, the reference's behaviour).
template <class CF, bool kWide>
__device__ __forceinline__ bool search_one(SearchCtx& c, ApfStage& apfs, AStarLdsT<CF>& alds, OuterLds* ol,
                                           long long hard_pops, bool resume, int dbg = 0, PrepL* pr = nullptr) {
  bind_hot<!kWide>(c);
  const PlannerDev& P = *c.P;
  const SlotArena& A = *c.A;
  const int lane = c.lane;
#ifdef HASTAR_STAMPS
  for (int q = 0; q < NSTAMP; ++q) c.cyc[q] = 0;
#endif
  unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  apf_stage(P, apfs, lane);
  if (kWide && pr) {  // a new epoch of the helper waves' prep table: this planner, its map and APF list
    c.prep_epoch += 1u;  // the main wave alone writes the epoch (and pidx, before the call): it counts its searches
    if (lane == 0) {
      prep_st(&pr->epoch, c.prep_epoch);
    }
    wave_lds_sync();
  }
  c.o3.t = c.open3;
  c.o3.lane = lane;
  c.o3.reset_cache();
  closed3_next_gen(c);
  c.status = 0;
  int counter = 0, interval = P.shot_interval;
  bool shot_allowed = false;
  uint64_t dig = 0x243f6a8885a308d3ull;
  int parks = 0;
  if (!resume) {
    c.n_closed3 = 0;
    c.pops = c.succ = c.apops = c.asearch = c.shots = c.amigr = c.apops_g = 0;
    c.ps3.next = 1;
    c.ps3.free = NIL;
    // Grid3D::set_start_node soft-resets the start cell's node (Grid3D.cpp:145-148 / 153-154)
    c.nm_f[(size_t)P.start_cx * c.N + P.start_cy] = euclid_h(P, P.start_cx, P.start_cy);
    Succ s0;
    s0.x = P.start_x;
    s0.y = P.start_y;
    s0.h = P.start_h;
    s0.g = 0.0f;
    s0.vmin = P.start_vmin;
    s0.ci = P.start_ci;
    s0.bin = P.start_bin;
    s0.cx = P.start_cx;
    s0.cy = P.start_cy;
    if (kWide && !(dbg & 1)) {  // the latency kernel starts in its LDS tree
      RBT<LdsAcc3> lt = lds_tree(*ol, c);
      lt.clear();
      insert3(c, lt, s0, FLT_MAX, NIL, OUTER_LDS_CAP);
    } else {
      c.o3.clear();
      insert3(c, c.o3, s0, FLT_MAX, NIL, A.open3_cap);
    }
  } else {
    // the loop state of the parked search; its open tree (header = node 0) and closed
    // records were copied into this arena by index
    const GAS SearchResult* R = gp(P.result);
    c.pops = R->pops;
    c.succ = R->successors;
    c.apops = R->astar_pops;
    c.asearch = R->astar_searches;
    c.shots = R->shots;
    c.amigr = R->astar_migrations;
    c.apops_g = R->astar_pops_hbm;
    dig = R->pop_digest;
    t_start = R->t_start;
    counter = R->counter;
    interval = R->interval;
    shot_allowed = R->shot_allowed != 0;
    c.n_closed3 = R->n_closed3;
    c.ps3.next = R->ps3_next;
    c.ps3.free = R->ps3_free;
    parks = R->parks;
    closed3_rebuild(c, c.n_closed3);
  }
  int ok = 0, via_shot = 0, terminal = NIL, dub_n = 0;
  float cost = FLT_MAX;
  // the planner's outer capacity after `parks` resumes (4x each), bounded by this arena: a
  // search parks at the same pop whatever arena the pool happens to hand it
  // (on the latency kernel, a head arena sized for the planner's known longest search, pops_grant,
  // lifts it: hastar_capi.cpp head_acquire.  Only that kernel gets head arenas; the batch kernel's
  // code stays as it was: an unused branch there moved its register allocation and cost 4 %)
  long long prule = (long long)P.arena_pops << (2 * min(parks, 12));
  if constexpr (kWide) prule = max(prule, (long long)A.pops_grant);
  const long long pcap = min(prule, (long long)SLOT3_IDX_MASK - 1);
  const int closed_lim = (int)min((long long)A.closed3_cap, pcap + 1);
  const int open_lim = (int)min((long long)A.open3_cap, 2 + (long long)(P.span_alloc - 1) * pcap + 64);
  STAMP_T tloop = STAMP_NOW();

  LoopState S;
  S.counter = counter;
  S.interval = interval;
  S.shot_allowed = shot_allowed;
  S.dig = dig;
  S.ok = ok;
  S.via_shot = via_shot;
  S.terminal = terminal;
  S.dub_n = dub_n;
  S.cost = cost;
  int code = LOOP_MIGRATE;
  if constexpr (kWide) {
    // the latency kernel keeps the outer tree in LDS while it fits (a resumed search moves
    // its tree in when it does), then continues in HBM
    if ((!resume || lds_outer_load(c, *ol, lane)) && !(dbg & 1)) {
      RBT<LdsAcc3> lt = lds_tree(*ol, c);
      code = search_loop<CF, true, kWide>(c, lt, apfs, alds, S, hard_pops, closed_lim, open_lim, OUTER_LDS_CAP, pr);
      if (code == LOOP_MIGRATE) lds_outer_store(c, *ol, lane);
    }
  }
  if (code == LOOP_MIGRATE) {
    c.o3.reset_cache();
    code = search_loop<CF, false, kWide>(c, c.o3, apfs, alds, S, hard_pops, closed_lim, open_lim, A.open3_cap, pr);
  }
  const bool handoff = code == LOOP_HANDOFF;  // (batch kernel only) a latency wave takes it over
  const bool parked = code == LOOP_PARKED || handoff;
  if constexpr (!kWide) {
    if (!handoff) ho_withdraw(c);
  }
  counter = S.counter;
  interval = S.interval;
  shot_allowed = S.shot_allowed;
  dig = S.dig;
  ok = S.ok;
  via_shot = S.via_shot;
  terminal = S.terminal;
  dub_n = S.dub_n;
  cost = S.cost;
  STAMP_ADD(6, tloop);
  if (parked) {
    if (lane == 0) {
      GAS SearchResult* R = gp(P.result);
      R->pops = c.pops;
      R->successors = c.succ;
      R->astar_pops = c.apops;
      R->astar_searches = c.asearch;
      R->shots = c.shots;
      R->astar_migrations = (int)c.amigr;
      R->astar_pops_hbm = c.apops_g;
      R->pop_digest = dig;
      R->t_start = t_start;
      R->counter = counter;
      R->interval = interval;
      R->shot_allowed = shot_allowed ? 1 : 0;
      R->n_closed3 = c.n_closed3;
      R->ps3_next = c.ps3.next;
      R->ps3_free = c.ps3.free;
      // the next capacity step beyond this arena's (a head arena's grant may exceed several);
      // a handoff is no capacity step: the search continues in this arena with its capacity
      int np = parks + 1;
      if constexpr (kWide)
        while (np < 12 && ((long long)P.arena_pops << (2 * np)) <= pcap) ++np;
      R->parks = handoff ? parks : np;
      R->park_arena = c.slot;
      R->ok = 0;
      R->path_len = 0;
      R->status = handoff ? SEARCH_HANDOFF : SEARCH_PARKED;
    }
    wave_lds_sync();
    if (handoff) c.status = SEARCH_HANDOFF;  // the kernel publishes it (READY) and stops
    return true;
  }
  if (c.status != 0) ok = 0;

  // ---- reconstruct_path (HybridAStar.cpp:208-262) into out_xyh / out_curv
  STAMP_T trc = STAMP_NOW();
  int path_len = 0;
  if (ok) {
    int L = 0;
    for (int i = terminal; i != NIL; i = c.closed3[i].prev) {
      if (dub_n + L >= P.out_cap || L >= A.chain_cap) { c.status = -28; break; }
      if (lane == 0) gp(A.out_chain)[L] = i;
      ++L;
    }
    wave_lds_sync();
    if (c.status == 0) {
      const float cs = P.rot_c, sn = P.rot_s, ang = -P.grid_heading;
      path_len = dub_n + L;
      for (int k = lane; k < path_len; k += 64) {
        float px, py, ph, kc = 0.0f;
        bool has_curv = true;
        if (k < dub_n) {
          const int q = dub_n - 1 - k;
          px = gp(A.dub_xyh)[3 * q];
          py = gp(A.dub_xyh)[3 * q + 1];
          ph = gp(A.dub_xyh)[3 * q + 2];
          kc = gp(A.dub_curv)[q];
        } else {
          const int m = k - dub_n;
          const Closed3 nd = gload(&c.closed3[gp(A.out_chain)[m]]);
          px = nd.x;
          py = nd.y;
          ph = nd.h;
          kc = gp(P.curv_abs)[nd.ci];
          has_curv = (m < L - 1);
        }
        const float x0 = px - P.goal_x, y0 = py - P.goal_y;
        float xr = x0 * cs + y0 * sn;
        float yr = -x0 * sn + y0 * cs;
        const float hr = wrap_pi_f(ph - ang);
        xr += P.world_goal_x;
        yr += P.world_goal_y;
        gp(P.out_xyh)[3 * k] = xr;
        gp(P.out_xyh)[3 * k + 1] = yr;
        gp(P.out_xyh)[3 * k + 2] = hr;
        if (has_curv) gp(P.out_curv)[k + 1] = kc;
      }
      if (lane == 0) gp(P.out_curv)[0] = 0.0f;
    } else {
      ok = 0;
    }
  }

  // ---- statistics: closed-set digest (order independent) and counters
  uint64_t cd = 0;
  for (int i = lane; i < c.n_closed3; i += 64) cd += mix64(digest_key(c.closed3[i].key));
  cd = wave_sum_u64(cd);
  wave_lds_sync();
  STAMP_ADD(5, trc);
  if (lane == 0) {
    auto R = gp(P.result);
    R->pops = c.pops;
    R->successors = c.succ;
    R->astar_pops = c.apops;
    R->astar_searches = c.asearch;
    R->shots = c.shots;
    R->closed_size = c.n_closed3;
    R->pop_digest = dig;
    R->closed_digest = cd;
    R->ok = ok;
    R->via_shot = via_shot;
    R->status = c.status;
    R->path_len = ok ? path_len : 0;
    R->cost = ok ? cost : FLT_MAX;
    R->terminal = terminal;
    R->dubins_len = dub_n;
    R->astar_migrations = c.amigr;
    R->astar_pops_hbm = c.apops_g;
    R->t_start = t_start;
    R->t_end = __builtin_amdgcn_s_memrealtime();
    R->slot = c.slot;
    // placement of the wave that ran it (diagnostics of the split launch):
    // s_getreg of HW_REG_XCC_ID (hwreg 20) and HW_REG_HW_ID (hwreg 4), full 32-bit fields
    R->hw_id = (int)(((uint32_t)__builtin_amdgcn_s_getreg(0xF814) & 0xfu) << 16 |
                     ((uint32_t)__builtin_amdgcn_s_getreg(0xF804) & 0xffffu));
    R->parks = parks;
#ifdef HASTAR_STAMPS
    c.cyc[22] = c.o3.n_fill;
    c.cyc[23] = c.o3.n_step;
    c.cyc[26] = c.o3.fill_cyc;
    c.cyc[27] = c.o3.pre_wait_cyc;
    c.cyc[28] = c.o3.pw_cyc;
    c.cyc[29] = c.o3.pw_ins_cyc;
    for (int q = 0; q < NSTAMP; ++q) R->cycles[q] = c.cyc[q];
#else
    for (int q = 0; q < NSTAMP; ++q) R->cycles[q] = 0;
#endif
  }
  wave_lds_sync();
  return false;
}

// Persistent work-queue kernel: one workgroup of 8 independent search wavefronts per CU, each
// with its own 20 KB slice of the CU's LDS (the workgroup takes the CU's whole LDS, so a
// latency-kernel workgroup of a split launch can only land on a CU this kernel left free).
// Wave w of workgroup b is slot s = 8 b + w and runs in arena s (slots >= n_slots take no
// work); it pulls planner indices (in `order`, longest-expected-first when the host knows)
// from a device counter until the queue is drained, so early finishers take the next planner.
constexpr int BATCH_WAVES = 8;
__global__ __launch_bounds__(64 * BATCH_WAVES) __attribute__((amdgpu_waves_per_eu(HASTAR_WAVES_PER_EU)))
void hastar_search_kernel(const PlannerDev* __restrict__ descs, int n_planners, const SlotArena* __restrict__ arenas,
                          int n_slots, const int* __restrict__ order, int* __restrict__ next, long long hard_pops,
                          int n_prio, int arena_base, int head_wgs) {
  __shared__ ApfStage apfs[BATCH_WAVES];
  __shared__ AStarLdsT<NarrowA> alds[BATCH_WAVES];
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform
  // head_wgs > 0: workgroups 0 .. head_wgs - 1 are head workgroups whose wave 0 alone runs
  // (a CU to itself), starting with queue entry b (the counter starts at head_wgs); slots
  // 0 .. head_wgs - 1, then 8 per workgroup
  const int b = (int)blockIdx.x;
  const bool head = b < head_wgs;
  if (head && w > 0) return;
  const int slot = head ? b : head_wgs + (b - head_wgs) * BATCH_WAVES + w;
  if (slot >= n_slots) return;  // a whole wave: no arena for it
  SearchCtx c;
  c.A = arenas + slot;
  c.slot = arena_base + slot;
  const SlotArena& A = *c.A;
  c.lane = (int)(threadIdx.x & 63);
  c.cost_only = true;
  c.gen3 = gp(A.gens)[0];
  c.gen2 = gp(A.gens)[1];
  c.status = 0;
  GAS HandoffBoard* const hb = ho_board(c);  // a split launch's board: this wave counts as running
  if (hb != nullptr && c.lane == 0) atomicAdd((int*)&hb->bulk_active, 1);
  for (bool first = true;; first = false) {
    int q = 0;
    if (first && head) {
      q = b;
    } else {
      if (c.lane == 0) q = atomicAdd(next, 1);
      q = __builtin_amdgcn_readfirstlane(__shfl(q, 0, 64));
    }
    if (q >= n_planners) break;
    // the queue is ordered longest-expected-first; the head of it runs at raised issue
    // priority so the batch's stragglers are not slowed by the waves sharing their SIMD
    if (q < n_prio) __builtin_amdgcn_s_setprio(3);
    else __builtin_amdgcn_s_setprio(0);
    c.P = descs + order[q];
    // a parked search keeps its state in this wave's arena: the wave takes no more work (a
    // handed-over one too: the latency wave continues it in this arena)
    if (search_one<NarrowA, false>(c, apfs[w], alds[w], nullptr, hard_pops, false)) {
      if (c.status == SEARCH_HANDOFF) {
        // publish the parked state (arena records, SearchResult, the planner's maps) and the
        // planner: READY.  The latency wave copies the records out of this arena, which no
        // other search uses in this launch: the wave takes no more work
        if (c.lane == 0) ho_st((GAS uint32_t*)&hb->entry[c.slot].pidx, (uint32_t)order[q]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (c.lane == 0) ho_st(&hb->state[c.slot], HANDOFF_READY);
      }
      break;
    }
  }
  if (c.lane == 0) {
    gp(A.gens)[0] = c.gen3;
    gp(A.gens)[1] = c.gen2;
    if (hb != nullptr) atomicSub((int*)&hb->bulk_active, 1);
  }
}

// The latency kernel: one search per CU.  A workgroup is one wavefront that takes the CU's
// whole LDS (static, 163 KB: no other workgroup of any kernel fits beside it), so its search
// keeps the outer open tree in LDS (OuterLds), the holonomic A* a 2048-node LDS pool with its
// {prev, g} pairs (WideA), and the obstacle list, and its wave issues alone on its SIMD.  The
// same search code as the batch kernel (search_one), so results are identical by
// construction; used for batches no larger than the CU count (the replan loop's pairs, single
// queries) and for resumed searches.  Persistent over the same work queue as
// hastar_search_kernel; resume = 1: workgroup b continues parked planner order[b] in arena b.
template <class CF>
struct WideLdsT {
  ApfStage apfs;
  AStarLdsT<CF> alds;
  OuterLds ol;
  PrepShared prep;
};
using WideLds = WideLdsT<WideA>;
static_assert(sizeof(WideLds) <= 163840, "the latency kernel's LDS must fit one CU");
// Wave 0 runs the searches; waves 1 .. PREP_HELPERS precompute expansions for it (prep_helper).
constexpr int WIDE_WAVES = 1 + PREP_HELPERS;
// One wave copies `bytes` (a multiple of 16) of 16-B-aligned records, 4 x 16 B per lane in flight.
__device__ __forceinline__ void copy_records(GAS void* dst, const GAS void* src, size_t bytes, int lane) {
  GAS v4i* d = (GAS v4i*)dst;
  const GAS v4i* s = (const GAS v4i*)src;
  const size_t n = bytes / 16;
  size_t i = (size_t)lane;
  for (; i + 192 < n; i += 256) {
    const v4i a = s[i], b = s[i + 64], e = s[i + 128], f = s[i + 192];
    d[i] = a;
    d[i + 64] = b;
    d[i + 128] = e;
    d[i + 192] = f;
  }
  for (; i < n; i += 64) d[i] = s[i];
}

// Latency kernel of a split launch: claim the oldest search a batch-kernel wave offers
// (HandoffBoard) and wait for its wave to park it (READY).  Returns the entry (= the arena the
// search's state stays in), or -1: no offer, or the search ended before its wave saw the claim.
__device__ __forceinline__ int ho_claim(const SearchCtx& c, GAS HandoffBoard* hb) {
  if (ho_ld((GAS uint32_t*)&hb->posted) == 0u) return -1;
  const int n = min(hb->n, HANDOFF_CAP);
  uint64_t key = ~0ull;  // (offer time << 12 | entry) of this lane's oldest offer
  for (int i = c.lane; i < n; i += 64) {
    if (ho_ld(&hb->state[i]) == HANDOFF_POSTED) {
      const uint64_t k = (ho_ld64((GAS uint64_t*)&hb->entry[i].t_start) << 12) | (uint64_t)i;
      key = k < key ? k : key;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)key, o, 64), hi = __shfl_xor((uint32_t)(key >> 32), o, 64);
    const uint64_t k = ((uint64_t)hi << 32) | lo;
    key = k < key ? k : key;
  }
  const uint32_t klo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)key);
  const uint32_t khi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(key >> 32));
  if (klo == 0xffffffffu && khi == 0xffffffffu) return -1;
  const int i = (int)(klo & 4095u);
  GAS uint32_t* st = &hb->state[i];
  uint32_t got = 0;
  if (c.lane == 0) got = atomicCAS((uint32_t*)st, HANDOFF_POSTED, HANDOFF_CLAIMED);
  got = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)got, 0, 64));
  if (got != HANDOFF_POSTED) return -1;  // withdrawn or taken meanwhile
  if (c.lane == 0) atomicSub((int*)&hb->posted, 1);
  // the batch wave answers within 64 pops: READY (parked for us) or CANCELLED (it ended first)
  uint32_t v;
  for (;;) {
    v = (uint32_t)__builtin_amdgcn_readfirstlane((int)ho_ld(st));
    if (v != HANDOFF_CLAIMED) break;
    __builtin_amdgcn_s_sleep(16);
  }
  if (v != HANDOFF_READY) {
    if (c.lane == 0) atomicCAS((uint32_t*)st, HANDOFF_CANCELLED, HANDOFF_EMPTY);
    return -1;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return i;
}

template <class CF>
__global__ __launch_bounds__(64 * WIDE_WAVES) void hastar_search_wide_kernel(
    const PlannerDev* __restrict__ descs, int n_planners, const SlotArena* __restrict__ arenas,
    const int* __restrict__ order, int* __restrict__ next, long long hard_pops, int resume, int dbg, int arena_base,
    int first_static) {
  __shared__ WideLdsT<CF> W;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = (int)(threadIdx.x & 63);
  PrepL* const tbl = lp(&W.prep);
  PrepL* pr = tbl;
  if (wv == 0) {
    for (int e = lane; e < PREP_E; e += 64) pr->state[e] = 0u;
    if (lane == 0) {
      pr->tail = 0u;
      pr->epoch = 0u;
      pr->stop = 0u;
    }
  }
  __syncthreads();  // the only workgroup barrier: helpers start on an initialised table
  const bool prep_on = !(dbg & 4);  // HASTAR_WIDE_DBG bit 2: no helper waves (diagnostics)
  if (wv > 0) {
    if (prep_on) prep_helper(*pr, W.apfs, descs, wv, lane);
    return;
  }
  if (!prep_on) pr = nullptr;
  SearchCtx c;
  c.A = arenas + blockIdx.x;
  c.slot = arena_base + (int)blockIdx.x;
  const SlotArena& A = *c.A;
  c.lane = lane;
  c.cost_only = true;
  c.prep_epoch = 0u;
  c.gen3 = gp(A.gens)[0];
  c.gen2 = gp(A.gens)[1];
  if (resume) {
    if ((int)blockIdx.x < n_planners) {
      const int pi = order[blockIdx.x];
      c.P = descs + pi;
      if (lane == 0) tbl->pidx = pi;
      search_one<CF, true>(c, W.apfs, W.alds, &W.ol, hard_pops, true, dbg, pr);
    }
  } else {
    // first_static: workgroup b runs queue entry b first (the head of a longest-first queue
    // split over this kernel and the batch kernel, whose counter starts after the head)
    // a split launch's latency CU prefers a long search the batch kernel offers (HandoffBoard)
    // to a new one from the queue, and once the queue is drained it waits for offers while
    // batch-kernel waves still run (bounded: 30 s without one, so every wave reaches its end).
    // No progress depends on the two kernels being co-resident, which HIP does not promise:
    //  - bulk_active counts batch waves that have STARTED and not yet ended (the batch kernel's
    //    entry and exit); a batch wave not yet resident is not counted, so a latency wave that sees 0
    //    leaves (it gives up offers it could have taken, never waits for an absent wave);
    //  - the claimer's wait for READY / CANCELLED is on an offer a running batch wave posted,
    //    and that wave answers within 64 of its pops or at its search's end;
    //  - the 30-s bound only guards a batch wave that stopped counting itself out (a fault).
    // The host cannot signal the wait: it regains control only when both kernels have ended.
    GAS HandoffBoard* const hb = first_static ? gp(A.board) : nullptr;
    const bool handoffs = hb != nullptr && hb->enabled != 0;
    for (bool first = true;; first = false) {
      int q = 0, ho = -1;
      if (first && first_static) {
        q = (int)blockIdx.x;
      } else {
        if (handoffs) ho = ho_claim(c, hb);
        if (ho < 0) {
          if (c.lane == 0) q = atomicAdd(next, 1);
          q = __builtin_amdgcn_readfirstlane(__shfl(q, 0, 64));
          if (q >= n_planners && handoffs) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
              ho = ho_claim(c, hb);
              if (ho >= 0) break;
              if (__builtin_amdgcn_readfirstlane((int)ho_ld((GAS uint32_t*)&hb->bulk_active)) <= 0) break;
              if (__builtin_amdgcn_s_memrealtime() - t0 > 3000000000ull) break;
              __builtin_amdgcn_s_sleep(64);
            }
          }
          if (ho < 0 && q >= n_planners) break;
        }
      }
      int pi;
      if (ho >= 0) {
        // the handed-over search: its open-tree nodes and closed records (the parked state,
        // SearchResult) are copied by index into this wave's arena, as a host resume copies
        // them, and it continues here in resume mode
        pi = __builtin_amdgcn_readfirstlane((int)ho_ld((GAS uint32_t*)&hb->entry[ho].pidx));
        const GAS SlotArena* src = gp(hb->pool) + ho;
        const GAS SearchResult* R = gp(descs[pi].result);
        copy_records(gp(A.open3), gp(src->open3), (size_t)R->ps3_next * sizeof(Node3), lane);
        copy_records(gp(A.closed3), gp(src->closed3), (size_t)R->n_closed3 * sizeof(Closed3), lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every load of the batch arena is back
        if (lane == 0) {
          ho_st(&hb->state[ho], HANDOFF_COPIED);
          atomicAdd((int*)&hb->handoffs, 1);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // the copies before the search's loads
      } else {
        pi = order[q];
      }
      c.P = descs + pi;
      if (lane == 0) tbl->pidx = pi;
      if (search_one<CF, true>(c, W.apfs, W.alds, &W.ol, hard_pops, ho >= 0, dbg, pr)) break;
    }
  }
  if (c.lane == 0) {
    gp(A.gens)[0] = c.gen3;
    gp(A.gens)[1] = c.gen2;
    prep_st(&tbl->stop, 1u);  // the helpers leave their loop
  }
}

// ------------------------------------------------- AStar<float> on its own (AStar.h) --
// The holonomic search of planner *P outside a Hybrid A* search (the reference's AStar
// class, used by utils/astar/test_astar.cpp): mode bit 0 = memo test of the start
// (find_path(int, int), AStar.cpp:100-113), bit 1 = get_cost_only (memo exits and the
// memo write-back), bit 2 = return the closed-record chain from the goal's predecessor
// (reconstruct_path, AStar.cpp:189-205), as world coordinates: the goal's predecessor
// first, each ((x - gx) * res, (y - gy) * res) rotated by -heading plus the goal position.
__global__ __launch_bounds__(64) void k_astar_query(const PlannerDev* __restrict__ P, const SlotArena* __restrict__ arena,
                                                    int si, int sj, int mode, float gwx, float gwy, float rc, float rs,
                                                    float* out_cost, float* xy, int cap, int* out_n) {
  __shared__ AStarLdsT<NarrowA> alds;
  SearchCtx c;
  c.P = P;
  c.A = arena;
  c.lane = threadIdx.x;
  bind_hot(c);
  c.cost_only = (mode & 2) != 0;
  c.gen2 = gp(arena->gens)[1];
  c.asearch = c.apops = c.amigr = c.apops_g = 0;
  c.status = 0;
  const float r = holonomic(c, alds, si, sj, (mode & 1) != 0);
  int n = 0;
  if ((mode & 4) && r < FLT_MAX && c.status == 0) {
    const PlannerDev& Pd = *P;
    const GAS Cell2* cells = gp(arena->cell2);
    const int goal = Pd.goal_cx * Pd.N + Pd.goal_cy;
    // the predecessor chain of the goal's closed record (cell indices)
    int cur = cells[goal].prev;
    while (cur != NIL) {
      if (n >= cap || cur < 0 || cur >= Pd.N * Pd.N) {
        n = -1;
        break;
      }
      if (c.lane == 0) {
        const int dx = cur / Pd.N - Pd.goal_cx, dy = cur % Pd.N - Pd.goal_cy;
        const float x = (float)dx * Pd.res, y = (float)dy * Pd.res;
        xy[2 * n] = x * rc + y * rs + gwx;
        xy[2 * n + 1] = -x * rs + y * rc + gwy;
      }
      ++n;
      cur = cells[cur].prev;
    }
  }
  if (c.lane == 0) {
    *out_cost = c.status == 0 ? r : FLT_MAX;
    *out_n = c.status == 0 ? n : -2;
    gp(arena->gens)[1] = c.gen2;
  }
}
hipError_t launch_astar_query(const PlannerDev* d_desc, const SlotArena* d_arena, int si, int sj, int mode, float gwx,
                              float gwy, float rc, float rs, float* out_cost, float* xy, int cap, int* out_n,
                              hipStream_t st) {
  hipLaunchKernelGGL(k_astar_query, dim3(1), dim3(64), 0, st, d_desc, d_arena, si, sj, mode, gwx, gwy, rc, rs, out_cost,
                     xy, cap, out_n);
  return hipGetLastError();
}

// ------------------------------------------------------ Grid3D<float> on its own ------
// Grid3D::get_neighbors (Grid3D.cpp:47-74) of one node: VehicleModel successors
// (VehicleModel.cpp:63-105) kept when their truncated cell is inside the grid and below the
// occupancy threshold, each with the APF field added to g and f (Grid3D.cpp:206-227).
// out: the kept successors (x, y, heading, g, vmin_sqr | curvature index, bin), cells: their
// (i, j); *count, *neglect = the model's returned flag.  One wavefront.
__global__ __launch_bounds__(64) void k_grid3d_neighbors(const PlannerDev* __restrict__ Pp, float nx, float ny, float nh,
                                                         float ng, float nvm, int nci, int nbin, float* out, int* cells,
                                                         int cap, int* count, int* neglect) {
  __shared__ ApfStage apfs;
  const PlannerDev& P = *Pp;
  const int lane = threadIdx.x;
  apf_stage(P, apfs, lane);
  wave_lds_sync();
  int lo = nci - P.na;
  lo = lo < 0 ? 0 : lo;
  const bool slow = nvm < 1.0f;
  int c = 0;
  for (int a = lo; a < lo + 2 * P.na + 1 && a < P.nsteer; ++a) {
    float vm = 0.0f;
    if (!slow) {
      const float lat = nvm * gp(P.curv_abs)[a];
      if (lat > P.a_lat) continue;
      const float al = (float)sqrt(1.0 - (double)((lat * lat) / P.a_lat2));
      vm = nvm - 2.0f * al * P.ts;
    }
    const GAS float* ofs = &gp(P.off)[2 * ((size_t)a * (P.bins + 1) + nbin)];
    const float sx = nx + ofs[0], sy = ny + ofs[1];
    const float sh = wrap_pi_f(nh + gp(P.dth)[a]);
    const int cx = trunc_f(sx / P.res), cy = trunc_f(sy / P.res);
    if (!(cx > -1 && cx < P.N && cy > -1 && cy < P.N)) continue;
    if (!(gp(P.occ)[(size_t)cx * P.N + cy] < P.thr)) continue;
    const float fc = apf_field(P, apfs, sx, sy, sh, lane);
    if (lane == 0 && c < cap) {
      const float g = ng + gp(P.act_cost)[a];
      float* o = out + 7 * c;
      o[0] = sx;
      o[1] = sy;
      o[2] = sh;
      o[3] = g + fc;  // _cost_g += field (Grid3D.cpp:66-67)
      o[4] = vm;
      o[5] = __int_as_float(a);
      o[6] = __int_as_float(heading_bin(sh, P.prec));
      cells[2 * c] = cx;
      cells[2 * c + 1] = cy;
    }
    ++c;
  }
  if (lane == 0) {
    *count = c;
    *neglect = slow ? 1 : 0;
  }
}
// Grid3D::check_path (Grid3D.cpp:78-93) of one sampled path
__global__ __launch_bounds__(64) void k_grid3d_check_path(const PlannerDev* __restrict__ Pp, const float* xyh, int n,
                                                          int* is_free) {
  const bool ok = path_is_free(*Pp, gp(xyh), n, threadIdx.x);
  if (threadIdx.x == 0) *is_free = ok ? 1 : 0;
}
hipError_t launch_grid3d_neighbors(const PlannerDev* d_desc, const float node[5], int nci, int nbin, float* out,
                                   int* cells, int cap, int* count, int* neglect, hipStream_t st) {
  hipLaunchKernelGGL(k_grid3d_neighbors, dim3(1), dim3(64), 0, st, d_desc, node[0], node[1], node[2], node[3], node[4],
                     nci, nbin, out, cells, cap, count, neglect);
  return hipGetLastError();
}
hipError_t launch_grid3d_check_path(const PlannerDev* d_desc, const float* xyh, int n, int* is_free, hipStream_t st) {
  hipLaunchKernelGGL(k_grid3d_check_path, dim3(1), dim3(64), 0, st, d_desc, xyh, n, is_free);
  return hipGetLastError();
}

// ------------------------------------------------------------------ map kernels -------
// Grid2D ctor + compute_heuristic (Grid2D.cpp:7-62, 303-316): _node_map f = h.
// Batched result hand-back: planner i's path (len_i points, when it fits the caller's
// buffer) is packed at point offset off[i] of one staging buffer, so a batch returns
// with a single device-to-host copy.
__global__ __launch_bounds__(256) void k_gather_paths(const PlannerDev* __restrict__ descs,
    const long long* __restrict__ off, const int* __restrict__ len, float* __restrict__ xyh, float* __restrict__ curv) {
  const int i = blockIdx.x;
  const int n = len[i];
  const long long o = off[i];
  const GAS float* sx = gp(descs[i].out_xyh);
  const GAS float* sc = gp(descs[i].out_curv);
  for (int t = threadIdx.x; t < 3 * n; t += blockDim.x) xyh[3 * o + t] = sx[t];
  for (int t = threadIdx.x; t < n; t += blockDim.x) curv[o + t] = sc[t];
}

// AStar::reset (AStar.cpp:56-60) of many planners: clear their visited bitmaps
// (ptrs: n bitmap pointers, words: 32-bit words per bitmap, a multiple of 4)
__global__ __launch_bounds__(256) void k_clear_bitmaps(uint32_t* const* __restrict__ ptrs, int n, size_t words) {
  for (int p = blockIdx.x; p < n; p += gridDim.x) {
    uint4* w = reinterpret_cast<uint4*>(ptrs[p]);
    for (size_t t = threadIdx.x; t < words / 4; t += blockDim.x) w[t] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// Grid2D ctor (Grid2D.cpp:7-62) + compute_heuristic (303-316): f plane = Euclidean h of every
// cell.  One workgroup per row (grid-strided): the row term dx² is computed once and the
// columns are written coalesced; no 64-bit divide per cell.  Same float expression as
// euclid_h, so the values are bit-identical.
__global__ __launch_bounds__(256) void k_init_nodemap(PlannerDev P) {
  const int N = P.N;
  GAS float* f = gp(P.nm_f);
  for (int i = blockIdx.x; i < N; i += gridDim.x) {
    const float dx = (float)(P.n45 - i) * P.res;
    const float dx2 = dx * dx;
    GAS float* row = f + (size_t)i * N;
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      const float dy = (float)(P.n2 - j) * P.res;
      const float dy2 = dy * dy;
      row[j] = sqrtf(dx2 + dy2);
    }
  }
}

// the same for n planners whose f planes lie `stride` bytes apart (hastar_create_batch_f32)
__global__ __launch_bounds__(256) void k_init_nodemap_batch(PlannerDev P, char* base, size_t stride, int n) {
  const int N = P.N;
  for (int pl = blockIdx.y; pl < n; pl += gridDim.y) {
    GAS float* f = gp(reinterpret_cast<float*>(base + stride * (size_t)pl));
    for (int i = blockIdx.x; i < N; i += gridDim.x) {
      const float dx = (float)(P.n45 - i) * P.res;
      const float dx2 = dx * dx;
      GAS float* row = f + (size_t)i * N;
      for (int j = threadIdx.x; j < N; j += blockDim.x) {
        const float dy = (float)(P.n2 - j) * P.res;
        const float dy2 = dy * dy;
        row[j] = sqrtf(dx2 + dy2);
      }
    }
  }
}
hipError_t launch_init_nodemap_batch(const PlannerDev& P, char* base, size_t stride, int n, hipStream_t st) {
  if (P.N <= 0 || n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_init_nodemap_batch, dim3(std::min(P.N, 256), std::min(n, 65535)), dim3(256), 0, st, P, base,
                     stride, n);
  return hipGetLastError();
}

// Grid2D::update_obstacles() (Grid2D.cpp:197-208), float4-vectorised.  `occ` may start
// anywhere (a row window of the map, see hastar_set_row_window): the cells before the first
// 16-B boundary and after the last one are done one by one.
__global__ void k_decay(float* __restrict__ occ, size_t NN, float lp_free, float lp_min, float lp_max) {
  const size_t mis = (size_t)((4 - ((reinterpret_cast<uintptr_t>(occ) >> 2) & 3)) & 3);
  const size_t head = mis < NN ? mis : NN;
  const size_t n4 = (NN - head) / 4;
  float4* o4 = reinterpret_cast<float4*>(occ + head);
  const size_t t0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x, dt = (size_t)gridDim.x * blockDim.x;
  for (size_t t = t0; t < n4; t += dt) {
    float4 v = o4[t];
    v.x = stl_max(stl_min(v.x + lp_free, lp_max), lp_min);
    v.y = stl_max(stl_min(v.y + lp_free, lp_max), lp_min);
    v.z = stl_max(stl_min(v.z + lp_free, lp_max), lp_min);
    v.w = stl_max(stl_min(v.w + lp_free, lp_max), lp_min);
    o4[t] = v;
  }
  if (t0 < head) occ[t0] = stl_max(stl_min(occ[t0] + lp_free, lp_max), lp_min);
  for (size_t t = head + n4 * 4 + t0; t < NN; t += dt)
    occ[t] = stl_max(stl_min(occ[t] + lp_free, lp_max), lp_min);
}

// Grid2D::update_obstacles(boxes) (Grid2D.cpp:99-139).  Boxes are applied in order (one
// workgroup walks them); inside one box every sub-sample adds the same delta and clamps,
// so a cell hit m times gets that step m times — counted with atomics, applied once per
// cell.  rp: per box {start_i, start_j, 2*end_i, 2*end_j}; dl: per box delta.
// Boxes of one "layer" (no two of them touch a common cell; the host orders layers so
// that overlapping boxes are applied in the reference's index order): one workgroup per
// box.  Within a box every sub-sample applies the same update, so counting the hits per
// cell and applying them m times in a row equals the reference's sequential loop.
__global__ __launch_bounds__(256) void k_raster_boxes(float* __restrict__ occ, int* __restrict__ cnt, int N,
                                                      const int* __restrict__ rp, const float* __restrict__ dl,
                                                      const int* __restrict__ ids, int nid, float c, float s,
                                                      float lp_min, float lp_max, int r0, int r1) {
  for (int q = blockIdx.x; q < nid; q += gridDim.x) {
    const int k = ids[q];
    const int si = rp[4 * k], sj = rp[4 * k + 1], ni = rp[4 * k + 2], nj = rp[4 * k + 3];
    const float d = dl[k];
    const int total = ni * nj;
    for (int pass = 0; pass < 2; ++pass) {
      for (int t = threadIdx.x; t < total; t += blockDim.x) {
        const int i = t / nj, j = t % nj;
        const float x0 = (float)(i * 0.5), y0 = (float)(j * 0.5);
        const float x = x0 * c + y0 * s;
        const float y = -x0 * s + y0 * c;
        const int ip = si + trunc_f(roundf(x)), jp = sj + trunc_f(roundf(y));
        if (ip >= r0 && ip < r1 && jp > -1 && jp < N) {
          const size_t cell = (size_t)ip * N + jp;
          if (pass == 0) {
            atomicAdd(&cnt[cell], 1);
          } else {
            const int m = atomicExch(&cnt[cell], 0);
            float v = occ[cell];
            for (int r = 0; r < m; ++r) {
              v += d;
              v = stl_max(stl_min(v, lp_max), lp_min);
            }
            if (m) occ[cell] = v;
          }
        }
      }
      __syncthreads();
    }
  }
}

// ---- batched map updates: many planners' maps per launch (hastar_*_batch) ----------
// Grid2D::update_obstacles() (Grid2D.cpp:197-208) of every map window of the batch:
// blockIdx.y walks the items, blockIdx.x strides through one window (float4 where aligned).
__device__ __forceinline__ float decay1(float v, float fr, float mn, float mx) {
  return stl_max(stl_min(v + fr, mx), mn);
}
__global__ __launch_bounds__(256) void k_decay_batch(const DecayItem* __restrict__ items, int n) {
  for (int q = blockIdx.y; q < n; q += gridDim.y) {
    const DecayItem it = items[q];
    float* occ = it.occ;
    const size_t NN = (size_t)it.cells;
    const size_t mis = (size_t)((4 - ((reinterpret_cast<uintptr_t>(occ) >> 2) & 3)) & 3);
    const size_t head = mis < NN ? mis : NN;
    const size_t n4 = (NN - head) / 4;
    float4* o4 = reinterpret_cast<float4*>(occ + head);
    const size_t t0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x, dt = (size_t)gridDim.x * blockDim.x;
    for (size_t t = t0; t < n4; t += dt) {
      float4 v = o4[t];
      v.x = decay1(v.x, it.lp_free, it.lp_min, it.lp_max);
      v.y = decay1(v.y, it.lp_free, it.lp_min, it.lp_max);
      v.z = decay1(v.z, it.lp_free, it.lp_min, it.lp_max);
      v.w = decay1(v.w, it.lp_free, it.lp_min, it.lp_max);
      o4[t] = v;
    }
    if (t0 < head) occ[t0] = decay1(occ[t0], it.lp_free, it.lp_min, it.lp_max);
    for (size_t t = head + n4 * 4 + t0; t < NN; t += dt) occ[t] = decay1(occ[t], it.lp_free, it.lp_min, it.lp_max);
  }
}

// Grid3D::relocate_obstacles (Grid3D.cpp:169-203) of every map of a chunk: claim pass (last
// writer = largest linear source index wins, as in the reference's row-major loop), gather
// into the map's scratch, copy back.
__global__ __launch_bounds__(256) void k_relocate_claim_batch(const RelocItem* __restrict__ items, int n) {
  for (int q = blockIdx.y; q < n; q += gridDim.y) {
    const RelocItem it = items[q];
    const int N = it.N;
    const size_t NN = (size_t)N * N;
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < NN; t += (size_t)gridDim.x * blockDim.x) {
      const float fi = (float)(int)(t / N), fj = (float)(int)(t % N);
      float x = fi * it.c + fj * it.s;
      float y = -fi * it.s + fj * it.c;
      x = x + it.ox;
      y = y + it.oy;
      const int a = trunc_f(roundf(x)), b = trunc_f(roundf(y));
      if (a > -1 && a < N && b > -1 && b < N) atomicMax(&it.winner[(size_t)a * N + b], (int)t);
    }
  }
}
__global__ __launch_bounds__(256) void k_relocate_gather_batch(const RelocItem* __restrict__ items, int n) {
  for (int q = blockIdx.y; q < n; q += gridDim.y) {
    const RelocItem it = items[q];
    const size_t NN = (size_t)it.N * it.N;
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < NN; t += (size_t)gridDim.x * blockDim.x) {
      const int w = it.winner[t];
      it.tmp[t] = (w >= 0) ? it.occ[w] : 0.0f;
      it.winner[t] = -1;
    }
  }
}
// ---- relocation by inversion (round 6): no claim table, no atomics ----------------------
// Every DESTINATION cell finds its winning source itself: the relocation is a rotation by
// (c, s) plus an offset, so the sources that round to destination (a, b) lie in the preimage
// of the unit square around (a, b), a unit square around the inverse-rotated point
// (i*, j*) = R^-1 ((a, b) - o) — within 0.7071 of it per axis, i.e. among the at most 2 x 2
// lattice points with |i - i*| <= 0.75 and |j - j*| <= 0.75.  Each candidate is tested with the
// reference's own forward arithmetic (the claim kernel's float expression), and the largest
// linear source index among the hits wins: the reference's row-major loop writes
// obstacle_map_new[i_new][j_new] last for the largest i * N + j (Grid3D.cpp:187-197).  The
// float inverse only chooses candidates (its error, below 1e-3 cell for coordinates under 1e4,
// is far inside the 0.043 margin); the forward test decides.  It compares in the float domain:
// static_cast<int>(std::round(x)) == a for a destination a >= 0 holds exactly when
// a - 0.5 <= x < a + 0.5 (a >= 1) or -0.5 < x < 0.5 (a = 0) — round half away from zero, and
// a +- 0.5 is exact in float — which is what trunc_f(roundf(x)) == a computes.
// The gather writes the relocated map into scratch (a destination may take its value from any
// cell of the old map), and k_relocate_copy_batch copies it back.
// The 2 x 2 candidates share their products: (i0, i0 + 1) * c and * s, (j0, j0 + 1) * s and * c
// as packed pairs (v_pk_mul_f32 / v_pk_add_f32 round each lane as the scalar ops do, and
// -ffp-contract=off keeps every product and sum separately rounded), the tests are evaluated
// branch-free, and the largest hit in row-major order (i0, j0) < (i0, j0 + 1) < (i0 + 1, j0) <
// (i0 + 1, j0 + 1) is selected.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int reloc_winner(int a, int b, int N, float c, float s, float ox, float oy) {
  const float fa = (float)a, fb = (float)b;
  const float dx = fa - ox, dy = fb - oy;
  const float is = dx * c - dy * s, js = dx * s + dy * c;  // R^-1 (x - o), candidates only
  const float fi0 = ceilf(is - 0.75f), fj0 = ceilf(js - 0.75f);
  const int i0 = (int)fi0, j0 = (int)fj0;
  const f2v fi = {fi0, fi0 + 1.0f}, fj = {fj0, fj0 + 1.0f};  // exact: integers far below 2^24
  const f2v cc = {c, c}, ss = {s, s};
  const f2v ic = fi * cc, is2 = fi * ss, js2 = fj * ss, jc = fj * cc;
  const f2v oxx = {ox, ox}, oyy = {oy, oy};
  // x = fi * c + fj * s + ox, y = -fi * s + fj * c + oy, for dj = 0 and dj = 1 (lanes: di)
  const f2v x0 = (ic + (f2v){js2.x, js2.x}) + oxx, x1 = (ic + (f2v){js2.y, js2.y}) + oxx;
  const f2v y0 = ((f2v){jc.x, jc.x} - is2) + oyy, y1 = ((f2v){jc.y, jc.y} - is2) + oyy;
  const float alo = fa - 0.5f, ahi = fa + 0.5f, blo = fb - 0.5f, bhi = fb + 0.5f;
  const bool a0 = a == 0, b0 = b == 0;
  auto inx = [&](float x) { return ((x > alo) | (!a0 & (x == alo))) & (x < ahi); };
  auto iny = [&](float y) { return ((y > blo) | (!b0 & (y == blo))) & (y < bhi); };
  const bool vi0 = (unsigned)i0 < (unsigned)N, vi1 = (unsigned)(i0 + 1) < (unsigned)N;
  const bool vj0 = (unsigned)j0 < (unsigned)N, vj1 = (unsigned)(j0 + 1) < (unsigned)N;
  const bool h00 = vi0 & vj0 & inx(x0.x) & iny(y0.x), h01 = vi0 & vj1 & inx(x1.x) & iny(y1.x);
  const bool h10 = vi1 & vj0 & inx(x0.y) & iny(y0.y), h11 = vi1 & vj1 & inx(x1.y) & iny(y1.y);
  const int base = i0 * N + j0;
  return h11 ? base + N + 1 : h10 ? base + N : h01 ? base + 1 : h00 ? base : -1;
}
// Gather of every map of a chunk into its scratch, in 2-D tiles so that one wave's gather stays
// compact in the source: a wave owns an 8 x 8 destination block (its preimage, a rotated 8 x 8,
// touches ~11 source rows x 1-2 lines instead of the up to 64 lines of a 64-cell row segment),
// four waves side by side make a 32-wide row band (8 full 128-B lines written per pass), and a
// workgroup walks RELOC_TILE_ROWS / 8 such bands.  blockIdx.y walks the items; blockIdx.x is the
// tile, dealt so that the 8 XCDs (blocks b and b + 8 share one) each take a contiguous band of
// the map: tiles near each other — whose preimages overlap — share one L2.
constexpr int RELOC_TILE_ROWS = 32;
__global__ __launch_bounds__(256) void k_relocate_invert_batch(const RelocItem* __restrict__ items, int n) {
  const int lane = (int)threadIdx.x & 63, wave = (int)threadIdx.x >> 6;
  for (int q = blockIdx.y; q < n; q += gridDim.y) {
    const RelocItem it = items[q];
    const int N = it.N;
    const int tx = (N + 31) / 32, ty = (N + RELOC_TILE_ROWS - 1) / RELOC_TILE_ROWS;
    const int per_xcd = (int)gridDim.x / 8;  // gridDim.x is a multiple of 8
    const int tile = ((int)blockIdx.x & 7) * per_xcd + ((int)blockIdx.x >> 3);
    const int b = (tile % tx) * 32 + wave * 8 + (lane & 7);
    const int a_top = (tile / tx) * RELOC_TILE_ROWS + (lane >> 3);
    if (tile >= tx * ty || b >= N) continue;
#pragma unroll
    for (int r = 0; r < RELOC_TILE_ROWS; r += 8) {
      const int a = a_top + r;
      if (a < N) {
        const int src = reloc_winner(a, b, N, it.c, it.s, it.ox, it.oy);
        const float v = src >= 0 ? ((const GAS float*)it.occ)[src] : 0.0f;  // unclaimed: the fresh map's 0
        ((GAS float*)it.tmp)[(size_t)a * N + b] = v;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_relocate_copy_batch(const RelocItem* __restrict__ items, int n) {
  for (int q = blockIdx.y; q < n; q += gridDim.y) {
    const RelocItem it = items[q];
    const size_t n4 = (size_t)it.N * it.N / 4, NN = (size_t)it.N * it.N;
    const float4* s4 = reinterpret_cast<const float4*>(it.tmp);
    float4* d4 = reinterpret_cast<float4*>(it.occ);
    const size_t t0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x, dt = (size_t)gridDim.x * blockDim.x;
    for (size_t t = t0; t < n4; t += dt) d4[t] = s4[t];
    for (size_t t = n4 * 4 + t0; t < NN; t += dt) it.occ[t] = it.tmp[t];
  }
}

// Grid2D::update_obstacles(boxes) (Grid2D.cpp:99-139), one workgroup per box of one layer
// (boxes of a layer never share a cell of their map; layers run in the reference's box
// order).  Within a box every sub-sample applies the same clamped update, so the hits of a
// cell are counted (LDS counters over the box footprint) and applied m times in a row —
// the reference's sequential loop, with no device-wide scratch, so the boxes of many
// planners can share a launch.
__global__ __launch_bounds__(256) void k_raster_boxes_batch(const RasterMap* __restrict__ maps,
                                                            const RasterBox* __restrict__ boxes, int nbox) {
  __shared__ int hist[RASTER_HIST];
  for (int q = blockIdx.x; q < nbox; q += gridDim.x) {
    const RasterBox b = boxes[q];
    const RasterMap m = maps[b.map];
    const int cells = b.bw * b.bh;
    for (int t = threadIdx.x; t < cells; t += blockDim.x) hist[t] = 0;
    __syncthreads();
    const int total = b.ni * b.nj;
    for (int t = threadIdx.x; t < total; t += blockDim.x) {
      const int i = t / b.nj, j = t % b.nj;
      const float x0 = (float)(i * 0.5), y0 = (float)(j * 0.5);
      const float x = x0 * m.c + y0 * m.s;
      const float y = -x0 * m.s + y0 * m.c;
      const int ip = b.si + trunc_f(roundf(x)), jp = b.sj + trunc_f(roundf(y));
      if (ip >= m.r0 && ip < m.r1 && jp > -1 && jp < m.N) atomicAdd(&hist[(ip - b.bi0) * b.bh + (jp - b.bj0)], 1);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < cells; t += blockDim.x) {
      const int cnt = hist[t];
      if (cnt == 0) continue;
      const size_t cell = (size_t)(b.bi0 + t / b.bh) * m.N + (b.bj0 + t % b.bh);
      float v = m.occ[cell];
      for (int r = 0; r < cnt; ++r) {
        v += b.d;
        v = stl_max(stl_min(v, m.lp_max), m.lp_min);
      }
      m.occ[cell] = v;
    }
    __syncthreads();
  }
}

// scatter of a batch's staged float lists (APF obstacle lists) into the planners' buffers
__global__ __launch_bounds__(64) void k_copy_batch(const CopyItem* __restrict__ items, int n,
                                                   const float* __restrict__ src) {
  for (int q = blockIdx.x; q < n; q += gridDim.x) {
    const CopyItem it = items[q];
    for (int t = threadIdx.x; t < it.count; t += blockDim.x) it.dst[t] = src[it.src_off + t];
  }
}

// Grid2D::update_obstacles(lines) (Grid2D.cpp:142-194).  lp: per line {ax, ay, dx, dy,
// nx, ny, delta, n_len, n_wid}; seq_len / seq_wid: the reference's float-accumulated
// progress values (prog_length / prog_width) computed on the host.
__global__ __launch_bounds__(1024) void k_raster_lines(float* __restrict__ occ, int* __restrict__ cnt, int N, int n45,
                                                       int n2, float res, const float* __restrict__ lp,
                                                       const float* __restrict__ seq_len,
                                                       const float* __restrict__ seq_wid, int seq_stride, int nline,
                                                       float lp_min, float lp_max, int r0, int r1) {
  for (int k = 0; k < nline; ++k) {
    const float* L = lp + 9 * k;
    const float ax = L[0], ay = L[1], dx = L[2], dy = L[3], nx = L[4], ny = L[5], d = L[6];
    const int nlen = (int)L[7], nwid = (int)L[8];
    const float* sl = seq_len + (size_t)k * seq_stride;
    const int total = nlen * nwid;
    for (int pass = 0; pass < 2; ++pass) {
      for (int t = threadIdx.x; t < total; t += blockDim.x) {
        const int a = t / nwid, b = t % nwid;
        const float pl = sl[a], pw = seq_wid[b];
        const float cx = ax + dx * pl, cy = ay + dy * pl;
        const float p1x = cx + nx * pw, p1y = cy + ny * pw;
        const float p2x = cx - nx * pw, p2y = cy - ny * pw;
        const int i1 = trunc_f(roundf(p1x / res)) + n45, i2 = trunc_f(roundf(p2x / res)) + n45;
        const int j1 = trunc_f(roundf(p1y / res)) + n2, j2 = trunc_f(roundf(p2y / res)) + n2;
        for (int e = 0; e < 2; ++e) {
          const int ii = e ? i2 : i1, jj = e ? j2 : j1;
          if (ii >= r0 && ii < r1 && jj > -1 && jj < N) {
            const size_t cell = (size_t)ii * N + jj;
            if (pass == 0) {
              atomicAdd(&cnt[cell], 1);
            } else {
              const int m = atomicExch(&cnt[cell], 0);
              float v = occ[cell];
              for (int q = 0; q < m; ++q) {
                v += d;
                v = stl_max(stl_min(v, lp_max), lp_min);
              }
              if (m) occ[cell] = v;
            }
          }
        }
      }
      __syncthreads();
    }
  }
}

// ------------------------------------------------ VelocityGenerator (post-search) -----
// VelocityGenerator<float>::generate_velocity_profile (VelocityGenerator.cpp:19-84), one
// thread per path.  The three passes are sequential along a path, so the parallelism is
// across paths.  velocity_sqr lives in the output array and the pass carries its running
// value in a register; the backward pass reads v²[i-1] before it overwrites it with v.
// The reference's float expressions are kept: `1.0 - x` promotes to double, so the
// remaining-acceleration term is a double sqrt rounded to float; hypot is glibc's hypotf.
__device__ __forceinline__ float vg_step(const float* X, int a, int b) {
  return g_hypotf(X[3 * a] - X[3 * b], X[3 * a + 1] - X[3 * b + 1]);
}
__device__ __forceinline__ float vg_long_rem(float acc, float vsq, float k, float lat2) {
  const float lat = vsq * k;
  return (float)((double)acc * sqrt(1.0 - (double)((lat * lat) / lat2)));
}
__global__ __launch_bounds__(64) void k_velocity_profile(VelParams vp, int n, const long long* __restrict__ off,
                                                         const float* __restrict__ xyh, const float* __restrict__ curv,
                                                         const float* __restrict__ vel_init,
                                                         const float* __restrict__ vmax_curr,
                                                         const unsigned char* __restrict__ flags, float* vel,
                                                         unsigned char* __restrict__ feasible) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const long long o = off[p];
  const int P = (int)(off[p + 1] - o);
  if (P <= 0) {  // no path (a failed search of a batch): nothing to profile
    feasible[p] = 0;
    return;
  }
  const float* X = xyh + 3 * o;
  const float* K = curv + o;
  float* V = vel + o;
  const unsigned char fl = flags[p];
  float vmax = (fl & 1u) ? vp.coast_velocity : vp.max_velocity;
  vmax = stl_min(vmax, vmax_curr[p]);
  const float vmax2 = vmax * vmax;
  const float v0 = vel_init[p];
  // Each pass walks its path in blocks of U points: the block's inputs (positions,
  // curvatures, v² of the previous pass) are loaded first, so the dependent chain waits
  // for memory once per block instead of once per point.  The step lengths are
  // hypot(x[a] - x[b], y[a] - y[b]) in the reference's operand order.
  constexpr int U = 16;
  const int S = P - 1;  // iterations per pass
  // initial profile: lateral-acceleration limits and braking to the velocity cap
  float cur = v0 * v0;
  V[0] = cur;
  float mcur = cur;
  for (int b = 0; b < S; b += U) {  // i = b + u, pi = P-1-i; points pi and pi-1
    float xs[U + 1], ys[U + 1], ks[U + 1];
#pragma unroll
    for (int u = 0; u <= U; ++u) {
      const int pi = P - 1 - (b + u);
      const bool in = b + u <= S;
      xs[u] = in ? X[3 * pi] : 0.0f;
      ys[u] = in ? X[3 * pi + 1] : 0.0f;
      ks[u] = in ? K[pi] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b + u >= S) break;
      const float step = g_hypotf(xs[u + 1] - xs[u], ys[u + 1] - ys[u]);
      const float rem = vg_long_rem(vp.max_long_dec, cur, ks[u], vp.max_lat_acc_sqr);
      mcur = stl_max(mcur - 2.0f * rem * step, vmax2);
      cur = (ks[u + 1] != 0.0f) ? stl_min(vp.max_lat_acc / ks[u + 1], mcur) : mcur;
      V[b + u + 1] = cur;
    }
  }
  if (fl & 2u) V[P - 1] = 0.0f;
  // forward pass (acceleration limit)
  cur = V[0];
  for (int b = 0; b < S; b += U) {
    float xs[U + 1], ys[U + 1], ks[U], vs[U];
#pragma unroll
    for (int u = 0; u <= U; ++u) {
      const int pi = P - 1 - (b + u);
      const bool in = b + u <= S;
      xs[u] = in ? X[3 * pi] : 0.0f;
      ys[u] = in ? X[3 * pi + 1] : 0.0f;
      if (u < U) {
        ks[u] = (b + u < S) ? K[pi] : 0.0f;
        vs[u] = (b + u < S) ? V[b + u + 1] : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b + u >= S) break;
      const float step = g_hypotf(xs[u + 1] - xs[u], ys[u + 1] - ys[u]);
      const float rem = vg_long_rem(vp.max_long_acc, cur, ks[u], vp.max_lat_acc_sqr);
      cur = stl_min(cur + 2.0f * rem * step, vs[u]);
      V[b + u + 1] = cur;
    }
  }
  // backward pass (braking limit), writing velocities: i = P-1 .. 1, pi = P-1-i = j
  cur = V[P - 1];
  const float last = cur;
  for (int b = 0; b < S; b += U) {  // j = b + u: points j and j+1, v² index i-1 = P-2-j
    float xs[U + 1], ys[U + 1], ks[U], vs[U];
#pragma unroll
    for (int u = 0; u <= U; ++u) {
      const int j = b + u;
      const bool in = j <= S;
      xs[u] = in ? X[3 * j] : 0.0f;
      ys[u] = in ? X[3 * j + 1] : 0.0f;
      if (u < U) {
        ks[u] = (j < S) ? K[j] : 0.0f;
        vs[u] = (j < S) ? V[P - 2 - j] : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (b + u >= S) break;
      const float step = g_hypotf(xs[u + 1] - xs[u], ys[u + 1] - ys[u]);
      const float rem = vg_long_rem(vp.max_long_dec, cur, ks[u], vp.max_lat_acc_sqr);
      cur = stl_min(cur + 2.0f * rem * step, vs[u]);
      V[P - 2 - (b + u)] = sqrtf(cur);
    }
  }
  V[P - 1] = sqrtf(last);
  feasible[p] = (v0 < (V[0] + 0.25f)) ? 1 : 0;
}

// ---------------------------------------------------------------- test kernels -------
__global__ void k_test_math(int fn, const float* a, const float* b, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = 0.0f;
  switch (fn) {
    case 0: v = g_sinf(a[i]); break;
    case 1: v = g_cosf(a[i]); break;
    case 2: v = g_atan2f(a[i], b[i]); break;
    case 3: v = g_acosf(a[i]); break;
    case 4: v = g_hypotf(a[i], b[i]); break;
    case 5: v = wrap_pi_f(a[i]); break;
    case 6: v = (float)heading_bin(a[i], b[i]); break;
    default: v = g_atanf(a[i]); break;
  }
  out[i] = v;
}

__global__ __launch_bounds__(64) void k_test_field(PlannerDev P, const float* poses, int n, float* out) {
  for (int q = blockIdx.x; q < n; q += gridDim.x) {
    __shared__ ApfStage apfs;
    apf_stage(P, apfs, threadIdx.x);
    const float f = apf_field(P, apfs, poses[3 * q], poses[3 * q + 1], poses[3 * q + 2], threadIdx.x);
    if (threadIdx.x == 0) out[q] = f;
  }
}

__global__ void k_test_dubins_len(float r, const float* starts, int n, float gx, float gy, float gh, float* out,
                                  int* word) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int w = 0;
  float prm[4];
  out[i] = dubins_shortest(r, starts[3 * i], starts[3 * i + 1], starts[3 * i + 2], gx, gy, gh, &w, prm);
  word[i] = w;
}

__global__ __launch_bounds__(64) void k_test_dubins_path(PlannerDev P, float sx, float sy, float sh, float* xyh,
                                                         float* curv, int cap, int* n_out, float* len_out,
                                                         int* flag_out) {
  int word = 0;
  float prm[4];
  const float len = dubins_shortest(P.r_min, sx, sy, sh, P.goal_x, P.goal_y, P.goal_h, &word, prm);
  const Centres C = dubins_centres(P.r_min, sx, sy, sh, P.goal_x, P.goal_y, P.goal_h);
  const int n = dubins_sample(P, C, word, prm, gp(xyh), gp(curv), cap, threadIdx.x);
  if (threadIdx.x == 0) {
    *n_out = n;
    *len_out = len;
    *flag_out = fabsf(prm[1]) > (float)M_PI_2;
  }
}

// ------------------------------------------------------------- launch wrappers -------
hipError_t launch_search(const PlannerDev* d_descs, int n, const SlotArena* d_arenas, int n_slots, const int* d_order, int n_prio,
                         int* d_next, long long hard_pops, hipStream_t st, int arena_base, int q0, int head_wgs) {
  // work counter q0 (>= 0: reset it; -1: the caller set it)
  if (head_wgs > 0) q0 = head_wgs;
  if (q0 >= 0) {
    const int init[4] = {q0, 0, 0, 0};
    hipError_t e = hipMemcpyAsync(d_next, init, sizeof(init), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
  }
  const int groups = head_wgs + (n_slots - head_wgs + BATCH_WAVES - 1) / BATCH_WAVES;
  hipLaunchKernelGGL(hastar_search_kernel, dim3(groups), dim3(64 * BATCH_WAVES), 0, st, d_descs, n, d_arenas, n_slots,
                     d_order, d_next, hard_pops, n_prio, arena_base, head_wgs);
  return hipGetLastError();
}
// HASTAR_WIDE_DBG (diagnostics): bit 0 keeps the latency kernel's outer tree in HBM, bit 2
// runs it without its helper waves
static int wide_dbg() {
  const char* e = std::getenv("HASTAR_WIDE_DBG");
  return e ? std::atoi(e) : 0;
}
static void launch_wide_cf(dim3 g, hipStream_t st, const PlannerDev* d, int n, const SlotArena* a, const int* o,
                           int* nx, long long hp, int resume, int dbg, int first_static = 0, int arena_base = 0) {
  hipLaunchKernelGGL(hastar_search_wide_kernel<WideA>, g, dim3(64 * WIDE_WAVES), 0, st, d, n, a, o, nx, hp, resume, dbg,
                     arena_base, first_static);
}
hipError_t launch_resume(const PlannerDev* d_descs, int n, const SlotArena* d_arenas, const int* d_order,
                         long long hard_pops, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  // a parked search is a long one: it continues on a CU of its own (the latency kernel)
  launch_wide_cf(dim3(n), st, d_descs, n, d_arenas, d_order, (int*)nullptr, hard_pops, 1, wide_dbg());
  return hipGetLastError();
}
hipError_t launch_search_wide(const PlannerDev* d_descs, int n, const SlotArena* d_arenas, int n_slots,
                              const int* d_order, int* d_next, long long hard_pops, hipStream_t st, int head,
                              int arena_base) {
  // head = 0: the whole queue (counter reset to 0); head = 1: the head of a split queue
  // (workgroup b takes entry b first; the caller set the counter past the head)
  if (!head) {
    const int init[4] = {0, 0, 0, 0};
    hipError_t e = hipMemcpyAsync(d_next, init, sizeof(init), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
  }
  launch_wide_cf(dim3(n_slots), st, d_descs, n, d_arenas, d_order, d_next, hard_pops, 0, wide_dbg(), head, arena_base);
  return hipGetLastError();
}
int search_slots_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, hastar_search_kernel, 64 * BATCH_WAVES, 0) != hipSuccess)
    return 1;
  return (nb > 0 ? nb : 1) * BATCH_WAVES;
}
hipError_t launch_gather_paths(const PlannerDev* d_descs, const long long* d_off, const int* d_len, int n, float* xyh,
                               float* curv, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_paths, dim3(n), dim3(256), 0, st, d_descs, d_off, d_len, xyh, curv);
  return hipGetLastError();
}
hipError_t launch_clear_bitmaps(uint32_t* const* ptrs, int n, size_t words, hipStream_t st) {
  hipLaunchKernelGGL(k_clear_bitmaps, dim3(std::min(n, 8192)), dim3(256), 0, st, ptrs, n, words);
  return hipGetLastError();
}
hipError_t launch_init_nodemap(const PlannerDev& P, hipStream_t st) {
  if (P.N <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_init_nodemap, dim3(std::min(P.N, 8192)), dim3(256), 0, st, P);
  return hipGetLastError();
}
hipError_t launch_decay(float* occ, size_t NN, float fr, float mn, float mx, hipStream_t st) {
  if (NN == 0) return hipSuccess;
  const int blocks = (int)((NN / 4 + 255) / 256 < 2048 ? (NN / 4 + 255) / 256 + 1 : 2048);
  hipLaunchKernelGGL(k_decay, dim3(blocks), dim3(256), 0, st, occ, NN, fr, mn, mx);
  return hipGetLastError();
}
hipError_t launch_raster_boxes(float* occ, int* cnt, int N, const int* rp, const float* dl, const int* ids, int nid,
                               float c, float s, float mn, float mx, int r0, int r1, hipStream_t st) {
  if (nid <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_raster_boxes, dim3(nid), dim3(256), 0, st, occ, cnt, N, rp, dl, ids, nid, c, s, mn, mx, r0, r1);
  return hipGetLastError();
}
hipError_t launch_raster_lines(float* occ, int* cnt, int N, int n45, int n2, float res, const float* lp,
                               const float* seq_len, const float* seq_wid, int stride, int nline, float mn, float mx,
                               int r0, int r1, hipStream_t st) {
  hipLaunchKernelGGL(k_raster_lines, dim3(1), dim3(1024), 0, st, occ, cnt, N, n45, n2, res, lp, seq_len, seq_wid,
                     stride, nline, mn, mx, r0, r1);
  return hipGetLastError();
}
static dim3 batch_grid(int n, size_t cells) {
  const size_t bx = std::min<size_t>((cells / 4 + 255) / 256 + 1, 256);
  return dim3((unsigned)bx, (unsigned)std::min(n, 65535));
}
hipError_t launch_decay_batch(const DecayItem* items, int n, size_t max_cells, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_decay_batch, batch_grid(n, max_cells), dim3(256), 0, st, items, n);
  return hipGetLastError();
}
// Relocation of n maps by inversion (k_relocate_invert_batch into each item's tmp, then
// k_relocate_copy_batch back): 16 N^2 bytes per map, no claim table.
hipError_t launch_relocate_invert(const RelocItem* items, int n, size_t max_cells, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int N = 1;
  while ((size_t)N * N < max_cells) ++N;
  // one workgroup per tile of the largest map, rounded up to a multiple of the 8 XCDs
  const size_t tiles = (size_t)((N + 31) / 32) * ((N + RELOC_TILE_ROWS - 1) / RELOC_TILE_ROWS);
  const unsigned bx = (unsigned)((tiles + 7) / 8 * 8);
  hipLaunchKernelGGL(k_relocate_invert_batch, dim3(bx, (unsigned)std::min(n, 65535)), dim3(256), 0, st, items, n);
  hipLaunchKernelGGL(k_relocate_copy_batch, batch_grid(n, max_cells), dim3(256), 0, st, items, n);
  return hipGetLastError();
}
hipError_t launch_relocate_batch(const RelocItem* items, int n, size_t max_cells, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const dim3 g = batch_grid(n, max_cells * 4);
  hipLaunchKernelGGL(k_relocate_claim_batch, g, dim3(256), 0, st, items, n);
  hipLaunchKernelGGL(k_relocate_gather_batch, g, dim3(256), 0, st, items, n);
  hipLaunchKernelGGL(k_relocate_copy_batch, batch_grid(n, max_cells), dim3(256), 0, st, items, n);
  return hipGetLastError();
}
hipError_t launch_raster_boxes_batch(const RasterMap* maps, const RasterBox* boxes, int nbox, hipStream_t st) {
  if (nbox <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_raster_boxes_batch, dim3(std::min(nbox, 65535)), dim3(256), 0, st, maps, boxes, nbox);
  return hipGetLastError();
}
hipError_t launch_copy_batch(const CopyItem* items, int n, const float* src, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_copy_batch, dim3(std::min(n, 65535)), dim3(64), 0, st, items, n, src);
  return hipGetLastError();
}
hipError_t launch_velocity_profile(const VelParams& vp, int n, const long long* off, const float* xyh, const float* curv,
                                   const float* vel_init, const float* vmax_curr, const unsigned char* flags, float* vel,
                                   unsigned char* feasible, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_velocity_profile, dim3((n + 63) / 64), dim3(64), 0, st, vp, n, off, xyh, curv, vel_init,
                     vmax_curr, flags, vel, feasible);
  return hipGetLastError();
}
hipError_t launch_test_math(int fn, const float* a, const float* b, float* out, int n, hipStream_t st) {
  hipLaunchKernelGGL(k_test_math, dim3((n + 255) / 256), dim3(256), 0, st, fn, a, b, out, n);
  return hipGetLastError();
}
hipError_t launch_test_field(const PlannerDev& P, const float* poses, int n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(k_test_field, dim3(n < 4096 ? n : 4096), dim3(64), 0, st, P, poses, n, out);
  return hipGetLastError();
}
hipError_t launch_test_dubins_len(float r, const float* starts, int n, float gx, float gy, float gh, float* out,
                                  int* word, hipStream_t st) {
  hipLaunchKernelGGL(k_test_dubins_len, dim3((n + 63) / 64), dim3(64), 0, st, r, starts, n, gx, gy, gh, out, word);
  return hipGetLastError();
}
hipError_t launch_test_dubins_path(const PlannerDev& P, float sx, float sy, float sh, float* xyh, float* curv,
                                   int cap, int* n_out, float* len_out, int* flag_out, hipStream_t st) {
  hipLaunchKernelGGL(k_test_dubins_path, dim3(1), dim3(64), 0, st, P, sx, sy, sh, xyh, curv, cap, n_out, len_out,
                     flag_out);
  return hipGetLastError();
}

}  // namespace hastar
