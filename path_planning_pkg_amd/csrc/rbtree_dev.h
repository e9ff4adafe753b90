// rbtree_dev.h — libstdc++-compatible red-black tree over an index pool, for HIP
// device code (also compiles for the host, used by the host-side unit test).
//
// The reference keeps its open sets in std::set<Node3D<T>> / std::set<Node2D<T>>
// (HybridAStar.h:72, AStar.h:70) with the comparator
//     a < b  <=>  a.key != b.key  &&  a.f < b.f          (Node3D.h:50-54, Node2D.h:41-45)
// which is not a strict weak ordering: whether an insert is dropped as a "duplicate" and
// which element find() returns depend on the exact path the lookup takes through the
// tree, i.e. on the tree SHAPE.  Reproducing the reference's search therefore requires
// libstdc++'s exact algorithms (GCC 11, bits/stl_tree.h + src/c++98/tree.cc):
//   _M_get_insert_unique_pos, _M_insert_ (insert_left rule), _M_lower_bound/find,
//   _Rb_tree_insert_and_rebalance, _Rb_tree_rebalance_for_erase, _Rb_tree_decrement.
// They are restated below on pool indices: node 0 is the header (p = root,
// l = leftmost, r = rightmost, color red), NIL (-1) is the null link.
// Tested against std::set on random operation streams: tools/rbtree_check.cpp, run by
// tests/test_capi_host.py.
#pragma once
#include <type_traits>
#include "hastar_layout.h"

#if defined(__HIPCC__)
#define RB_HD __host__ __device__ __forceinline__
#else
#define RB_HD inline
#endif

namespace hastar {

// Tree walks are wave-uniform (every lane follows the same path): on the device the
// loaded links/keys are moved to SGPRs so the walk compiles to scalar control flow.
#if defined(__HIPCC__)
__host__ __device__ __forceinline__ int rb_ui(int v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(v);
#else
  return v;
#endif
}
__host__ __device__ __forceinline__ uint32_t rb_uu(uint32_t v) { return (uint32_t)rb_ui((int)v); }
__host__ __device__ __forceinline__ float rb_uf(float v) { return __int_as_float(rb_ui(__float_as_int(v))); }
#else
inline int rb_ui(int v) { return v; }
inline uint32_t rb_uu(uint32_t v) { return v; }
inline float rb_uf(float v) { return v; }
#endif

// comparator of the reference: (ka != kb) && (fa < fb); FT = the planner's T (float, or
// double for HybridAStar<double>, hastar_f64.hip)
template <class FT>
RB_HD bool rb_less(uint32_t ka, FT fa, uint32_t kb, FT fb) { return (ka != kb) && (fa < fb); }

// {key, f, l, r} of one node (for float: one 16-byte load, the first 16 bytes of every node type)
template <class FT>
struct QuadT {
  uint32_t key;
  FT f;
  int l, r;
};
using Quad = QuadT<float>;

// the f type of a tree layout: Acc::FT when the accessor declares one, else float
template <class A, class = void>
struct rb_acc_ft {
  using type = float;
};
template <class A>
struct rb_acc_ft<A, std::void_t<typename A::FT>> {
  using type = typename A::FT;
};
#if defined(__HIP_DEVICE_COMPILE__)
typedef int rb_v4i __attribute__((ext_vector_type(4)));
template <class PtrT>
__device__ __forceinline__ Quad rb_quad(PtrT t, int x) {
  typedef typename std::remove_reference<decltype(t[0].key)>::type K;  // keeps the address space
  (void)sizeof(K);
  const rb_v4i v = *reinterpret_cast<decltype(&reinterpret_cast<const rb_v4i&>(t[x]))>(&t[x]);
  Quad q;
  q.key = rb_uu((uint32_t)v.x);
  q.f = __int_as_float(rb_ui(v.y));
  q.l = rb_ui(v.z);
  q.r = rb_ui(v.w);
  return q;
}
#else
template <class PtrT>
RB_HD Quad rb_quad(PtrT t, int x) {
  return Quad{t[x].key, t[x].f, t[x].l, t[x].r};
}
#endif

// Field access of a tree layout.  The algorithms below (RBT) only use these members,
// so the same libstdc++ restatement runs on the array-of-structs HBM nodes (Node3,
// Node2; 32-bit links) and on the compact LDS nodes of the inner A* (16-bit links).
template <class NodeT, class PtrT = NodeT*>
struct AosAcc {
  static constexpr bool kPathWalk = false;
  PtrT t;
  RB_HD int L(int x) const { return rb_ui(t[x].l); }
  RB_HD int R(int x) const { return rb_ui(t[x].r); }
  RB_HD int P(int x) const { return rb_ui(t[x].p); }
  RB_HD int C(int x) const { return rb_ui(t[x].color); }
  RB_HD void sL(int x, int v) { t[x].l = v; }
  RB_HD void sR(int x, int v) { t[x].r = v; }
  RB_HD void sP(int x, int v) { t[x].p = v; }
  RB_HD void sC(int x, int v) { t[x].color = v; }
  RB_HD uint32_t K(int x) const { return rb_uu(t[x].key); }
  RB_HD float F(int x) const { return rb_uf(t[x].f); }
  RB_HD Quad quad(int x) const { return rb_quad(t, x); }
  RB_HD Quad quad_at(int x, int depth) { return quad(x); }  // walk step at depth (cache hook)
  RB_HD void leaf(int x, int p) {  // new node: parent p, no children, red
    t[x].p = p;
    t[x].l = NIL;
    t[x].r = NIL;
    t[x].color = RB_RED;
  }
};

template <class Acc>
struct RBT : Acc {
  using Acc::L;
  using Acc::R;
  using Acc::P;
  using Acc::C;
  using Acc::sL;
  using Acc::sR;
  using Acc::sP;
  using Acc::sC;
  using Acc::K;
  using Acc::F;
  using FT = typename rb_acc_ft<Acc>::type;
  using Q = QuadT<FT>;

  RB_HD int root() { return P(0); }
  RB_HD int begin() { return L(0); }  // == 0 (header) when empty
  RB_HD bool empty() { return P(0) == NIL; }

  RB_HD void clear() {
    sP(0, NIL);
    sL(0, 0);
    sR(0, 0);
    sC(0, RB_RED);
  }

  RB_HD void rotate_left(int x) {
    const int y = R(x);
    const int yl = L(y);
    sR(x, yl);
    if (yl != NIL) sP(yl, x);
    const int xp = P(x);
    sP(y, xp);
    if (x == P(0)) sP(0, y);
    else if (x == L(xp)) sL(xp, y);
    else sR(xp, y);
    sL(y, x);
    sP(x, y);
  }

  RB_HD void rotate_right(int x) {
    const int y = L(x);
    const int yr = R(y);
    sL(x, yr);
    if (yr != NIL) sP(yr, x);
    const int xp = P(x);
    sP(y, xp);
    if (x == P(0)) sP(0, y);
    else if (x == R(xp)) sR(xp, y);
    else sL(xp, y);
    sR(y, x);
    sP(x, y);
  }

  RB_HD int decrement(int x) {
    if (C(x) == RB_RED && P(x) != NIL && P(P(x)) == x) return R(x);  // header
    if (L(x) != NIL) {
      int y = L(x);
      while (R(y) != NIL) y = R(y);
      return y;
    }
    int y = P(x);
    while (x == L(y)) {
      x = y;
      y = P(y);
    }
    return y;
  }

  // std::set::find (stl_tree.h _M_lower_bound + key_compare check).  Returns 0 (= end)
  // when not "found".
  RB_HD int find(uint32_t k, FT f) {
    int y = 0, x = P(0), depth = 0;
    uint32_t yk = 0;
    FT yf = 0;
    if constexpr (Acc::kPathWalk) {
      bool unused;
      int rj;
      uint32_t rk;
      FT rf;
      this->path_walk(k, f, false, &y, &yk, &yf, &unused, &rj, &rk, &rf);
      x = NIL;
    }
    while (x != NIL) {
      const Q q = this->quad_at(x, depth++);
      if (!rb_less(q.key, q.f, k, f)) {
        y = x;
        yk = q.key;
        yf = q.f;
        x = q.l;
      } else {
        x = q.r;
      }
    }
    if (y == 0 || rb_less(k, f, yk, yf)) return 0;
    return y;
  }

  // _M_get_insert_unique_pos: returns the parent for the new node (>= 0) or -2 when an
  // "equivalent" element exists (insert dropped).  *left = insert_left of _M_insert_.
  RB_HD int insert_pos(uint32_t k, FT f, bool* left) {
    int x = P(0), y = 0, depth = 0;
    bool comp = true;
    uint32_t yk = 0;
    FT yf = 0;
    if constexpr (Acc::kPathWalk) {
      // The walk also reports the deepest node where it turned right (rj; -1 if none).
      // That node is decrement(y) when the walk ended by going left, and y is the
      // leftmost node when it never turned right, so _M_get_insert_unique_pos needs no
      // further tree access.
      int rj;
      uint32_t rk;
      FT rf;
      this->path_walk(k, f, true, &y, &yk, &yf, &comp, &rj, &rk, &rf);
      if (comp) {
        if (rj < 0) {
          *left = true;  // y == L(0)
          return y;
        }
        if (rb_less(rk, rf, k, f)) {
          *left = (y == 0) || rb_less(k, f, yk, yf);
          return y;
        }
        return -2;
      }
      if (rb_less(yk, yf, k, f)) {
        *left = (y == 0) || rb_less(k, f, yk, yf);
        return y;
      }
      return -2;
    }
    while (x != NIL) {
      const Q q = this->quad_at(x, depth++);
      y = x;
      yk = q.key;
      yf = q.f;
      comp = rb_less(k, f, q.key, q.f);
      x = comp ? q.l : q.r;
    }
    int j = y;
    if (comp) {
      if (j == L(0)) {
        *left = true;  // _M_insert_: x != 0 is false; p == end() or comp(v, p) holds
        return y;
      }
      j = decrement(j);
    }
    if (rb_less(K(j), F(j), k, f)) {
      *left = (y == 0) || rb_less(k, f, yk, yf);
      return y;
    }
    return -2;
  }

  // _Rb_tree_insert_and_rebalance(insert_left, x, p, header)
  RB_HD void link(bool insert_left, int x, int p) {
    this->leaf(x, p);
    if (insert_left) {
      sL(p, x);
      if (p == 0) {
        sP(0, x);
        sR(0, x);
      } else if (p == L(0)) {
        sL(0, x);
      }
    } else {
      sR(p, x);
      if (p == R(0)) sR(0, x);
    }
    // xp = P(x) throughout; it is p after leaf(x, p), so the usual first iteration (x's new
    // parent black) reads no link at all.  rootv = P(0) is refreshed after every rotation, so it
    // is the root at the end.
    int rootv = P(0);
    int xp = p;
    while (x != rootv) {
      if (C(xp) != RB_RED) break;
      const int xpp = P(xp);
      if (xp == L(xpp)) {
        const int y = R(xpp);
        if (y != NIL && C(y) == RB_RED) {
          sC(xp, RB_BLACK);
          sC(y, RB_BLACK);
          sC(xpp, RB_RED);
          x = xpp;
        } else {
          if (x == R(xp)) {
            x = xp;
            rotate_left(x);
          }
          sC(P(x), RB_BLACK);
          sC(xpp, RB_RED);
          rotate_right(xpp);
          rootv = P(0);
        }
      } else {
        const int y = L(xpp);
        if (y != NIL && C(y) == RB_RED) {
          sC(xp, RB_BLACK);
          sC(y, RB_BLACK);
          sC(xpp, RB_RED);
          x = xpp;
        } else {
          if (x == L(xp)) {
            x = xp;
            rotate_right(x);
          }
          sC(P(x), RB_BLACK);
          sC(xpp, RB_RED);
          rotate_left(xpp);
          rootv = P(0);
        }
      }
      xp = P(x);
    }
    sC(rootv, RB_BLACK);
  }

  RB_HD int minimum(int x) {
    while (L(x) != NIL) x = L(x);
    return x;
  }
  RB_HD int maximum(int x) {
    while (R(x) != NIL) x = R(x);
    return x;
  }

  // _Rb_tree_rebalance_for_erase(z, header); the caller frees z afterwards.
  RB_HD void unlink(int z) {
    int y = z, x = NIL, xp = NIL;
    const int zl = L(z), zr = R(z), zp = P(z);
    if (zl == NIL) {
      x = zr;
    } else if (zr == NIL) {
      x = zl;
    } else {
      y = zr;
      while (L(y) != NIL) y = L(y);
      x = R(y);
    }
    if (y != z) {
      sP(zl, y);
      sL(y, zl);
      if (y != zr) {
        xp = P(y);
        if (x != NIL) sP(x, xp);
        sL(xp, x);
        sR(y, zr);
        sP(zr, y);
      } else {
        xp = y;
      }
      if (P(0) == z) sP(0, y);
      else if (L(zp) == z) sL(zp, y);
      else sR(zp, y);
      sP(y, zp);
      const int cy = C(y);
      sC(y, C(z));
      sC(z, cy);
      y = z;
    } else {
      xp = zp;
      if (x != NIL) sP(x, zp);
      if (P(0) == z) sP(0, x);
      else if (L(zp) == z) sL(zp, x);
      else sR(zp, x);
      if (L(0) == z) sL(0, (zr == NIL) ? zp : minimum(x));
      if (R(0) == z) sR(0, (zl == NIL) ? zp : maximum(x));
    }
    if (C(y) != RB_RED) {
      while (x != P(0) && (x == NIL || C(x) == RB_BLACK)) {
        if (x == L(xp)) {
          int w = R(xp);
          if (C(w) == RB_RED) {
            sC(w, RB_BLACK);
            sC(xp, RB_RED);
            rotate_left(xp);
            w = R(xp);
          }
          const int wl = L(w), wr = R(w);
          if ((wl == NIL || C(wl) == RB_BLACK) && (wr == NIL || C(wr) == RB_BLACK)) {
            sC(w, RB_RED);
            x = xp;
            xp = P(xp);
          } else {
            if (wr == NIL || C(wr) == RB_BLACK) {
              sC(wl, RB_BLACK);
              sC(w, RB_RED);
              rotate_right(w);
              w = R(xp);
            }
            sC(w, C(xp));
            sC(xp, RB_BLACK);
            if (R(w) != NIL) sC(R(w), RB_BLACK);
            rotate_left(xp);
            break;
          }
        } else {
          int w = L(xp);
          if (C(w) == RB_RED) {
            sC(w, RB_BLACK);
            sC(xp, RB_RED);
            rotate_right(xp);
            w = L(xp);
          }
          const int wl = L(w), wr = R(w);
          if ((wr == NIL || C(wr) == RB_BLACK) && (wl == NIL || C(wl) == RB_BLACK)) {
            sC(w, RB_RED);
            x = xp;
            xp = P(xp);
          } else {
            if (wl == NIL || C(wl) == RB_BLACK) {
              sC(wr, RB_BLACK);
              sC(w, RB_RED);
              rotate_left(w);
              w = L(xp);
            }
            sC(w, C(xp));
            sC(xp, RB_BLACK);
            if (L(w) != NIL) sC(L(w), RB_BLACK);
            rotate_right(xp);
            break;
          }
        }
      }
      if (x != NIL) sC(x, RB_BLACK);
    }
  }
};

template <class NodeT, class PtrT = NodeT*>
using RBTree = RBT<AosAcc<NodeT, PtrT>>;

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// Outer open tree: Node3 records in HBM behind a 64-entry, fully associative,
// write-through node cache held in the wavefront's registers.  Lane i caches the whole
// tree part of one node (id, key, f, l, r, p, color), so every accessor the libstdc++
// algorithms use (walks, link/rebalance, erase/rebalance, the pool's free list) costs a
// ballot and one lane read on a hit instead of a dependent HBM round trip.  A miss loads
// the node's first two quads (one round trip) and fills a lane.  Lanes 0..PATH-1 hold the
// root-to-leaf path of the last walk (lane d = the node at depth d), the header lives in
// lane 63, other misses rotate through lanes PATH..62.  Every tree write goes to HBM and
// to every lane caching that node, so the cache is never stale.
//
// Path walks: a new walk follows the cached path for as long as its own branch decision
// at depth d leads to the cached node at depth d + 1.  Every path lane evaluates that
// decision on its own node at once, so the shared prefix costs one ballot instead of a
// chain of dependent steps; the walk continues step by step only below the point where
// it leaves the cached path (consecutive inserts of similar f share most of it).
// All calls are wave-uniform.
struct CachedAcc3 {
  static constexpr bool kPathWalk = true;
  static constexpr int PATH = 48;
  __attribute__((address_space(1))) Node3* t;
  int lane;
  int cid;      // this lane's cached node (-1: empty)
  uint32_t ck;
  float cf;
  int cl, cr, cp;
  uint32_t cc;  // color (byte 0) | curvature index << 8
  float cg, cvm, cx, cy, ch;  // payload: g, vmin, pose
  int cpv;                    // payload: prev
  int rr;       // round-robin victim counter (wave-uniform)
  int plen;     // lanes [0, plen) hold the last walk's path (wave-uniform)
#ifdef HASTAR_STAMPS
  unsigned long long n_fill, n_step, fill_cyc, pre_wait_cyc, pw_cyc, pw_ins_cyc;  // diagnostics
#endif

  __device__ __forceinline__ void reset_cache() {
    cid = -1;
    rr = 0;
    plen = 0;
#ifdef HASTAR_STAMPS
    n_fill = n_step = fill_cyc = pre_wait_cyc = pw_cyc = pw_ins_cyc = 0;
#endif
  }
  __device__ __forceinline__ int hit(int x) const {
    const uint64_t m = __ballot(cid == x);
    return m ? (int)__ffsll((unsigned long long)m) - 1 : -1;
  }
  __device__ __forceinline__ int victim(int x) {
    if (x == 0) return 63;
    const int v = PATH + rr;
    rr = rr == 62 - PATH ? 0 : rr + 1;
    return v;
  }
  // lane `slot` takes node x from registers of lane `h` (h may be any lane)
  __device__ __forceinline__ void copy_from(int x, int h, int slot) {
    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)ck, h);
    const float f = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), h));
    const int l = __builtin_amdgcn_readlane(cl, h), r = __builtin_amdgcn_readlane(cr, h);
    const int p = __builtin_amdgcn_readlane(cp, h);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cc, h);
    const float g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cg), h));
    const float vm = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cvm), h));
    const float px = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cx), h));
    const float py = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cy), h));
    const float ph = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ch), h));
    const int pv = __builtin_amdgcn_readlane(cpv, h);
    if (lane == slot) {
      cid = x;
      ck = k;
      cf = f;
      cl = l;
      cr = r;
      cp = p;
      cc = c;
      cg = g;
      cvm = vm;
      cx = px;
      cy = py;
      ch = ph;
      cpv = pv;
    }
  }
  // one round trip: the whole 48-B record of node x, cached in lane `slot`; returns the
  // record as wave-uniform values
  __device__ __forceinline__ Node3 fill(int x, int slot) {
    typedef int v4 __attribute__((ext_vector_type(4)));
#ifdef HASTAR_STAMPS
    const unsigned long long ta = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    pre_wait_cyc += t0 - ta;
#endif
    const __attribute__((address_space(1))) v4* q = (const __attribute__((address_space(1))) v4*)&t[x];
    const v4 a = q[0], b = q[1], d = q[2];
#ifdef HASTAR_STAMPS
    n_fill++;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    // every lane loaded the same record: the cache lane takes the loaded vector registers
    // as they are; the wave-uniform copies below are only materialised (readfirstlane)
    // for the fields a caller actually uses (the rest is dead code after inlining)
    if (lane == slot) {
      cid = x;
      ck = (uint32_t)a.x;
      cf = __int_as_float(a.y);
      cl = a.z;
      cr = a.w;
      cp = b.x;
      cc = (uint32_t)b.y;
      cg = __int_as_float(b.z);
      cvm = __int_as_float(b.w);
      cx = __int_as_float(d.x);
      cy = __int_as_float(d.y);
      ch = __int_as_float(d.z);
      cpv = d.w;
    }
    Node3 n;
    n.key = rb_uu((uint32_t)a.x);
#ifdef HASTAR_STAMPS
    fill_cyc += __builtin_amdgcn_s_memtime() - t0;
#endif
    n.f = __int_as_float(rb_ui(a.y));
    n.l = rb_ui(a.z);
    n.r = rb_ui(a.w);
    n.p = rb_ui(b.x);
    n.cc = rb_uu((uint32_t)b.y);
    n.g = __int_as_float(rb_ui(b.z));
    n.vmin = __int_as_float(rb_ui(b.w));
    n.x = __int_as_float(rb_ui(d.x));
    n.y = __int_as_float(rb_ui(d.y));
    n.h = __int_as_float(rb_ui(d.z));
    n.prev = rb_ui(d.w);
    return n;
  }
  __device__ __forceinline__ void set_lane(int x, const Node3& n) {
    cid = x;
    ck = n.key;
    cf = n.f;
    cl = n.l;
    cr = n.r;
    cp = n.p;
    cc = n.cc;
    cg = n.g;
    cvm = n.vmin;
    cx = n.x;
    cy = n.y;
    ch = n.h;
    cpv = n.prev;
  }
  __device__ __forceinline__ int L(int x) {
    const int h = hit(x);
    return h >= 0 ? __builtin_amdgcn_readlane(cl, h) : fill(x, victim(x)).l;
  }
  __device__ __forceinline__ int R(int x) {
    const int h = hit(x);
    return h >= 0 ? __builtin_amdgcn_readlane(cr, h) : fill(x, victim(x)).r;
  }
  __device__ __forceinline__ int P(int x) {
    const int h = hit(x);
    return h >= 0 ? __builtin_amdgcn_readlane(cp, h) : fill(x, victim(x)).p;
  }
  __device__ __forceinline__ int C(int x) {
    const int h = hit(x);
    return (int)((h >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)cc, h) : fill(x, victim(x)).cc) & 0xffu);
  }
  __device__ __forceinline__ uint32_t K(int x) {
    const int h = hit(x);
    return h >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)ck, h) : fill(x, victim(x)).key;
  }
  __device__ __forceinline__ float F(int x) {
    const int h = hit(x);
    return h >= 0 ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), h)) : fill(x, victim(x)).f;
  }
  __device__ __forceinline__ float G(int x) {
    const int h = hit(x);
    return h >= 0 ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cg), h)) : fill(x, victim(x)).g;
  }
  // the whole record of node x (the pop reads the payload from the cache when it can)
  __device__ __forceinline__ Node3 node(int x) {
#ifdef HASTAR_DBG_NOPAY
    const int h = -1;
#else
    const int h = hit(x);
#endif
    if (h < 0) return fill(x, victim(x));
    Node3 n;
    n.key = (uint32_t)__builtin_amdgcn_readlane((int)ck, h);
    n.f = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), h));
    n.l = __builtin_amdgcn_readlane(cl, h);
    n.r = __builtin_amdgcn_readlane(cr, h);
    n.p = __builtin_amdgcn_readlane(cp, h);
    n.cc = (uint32_t)__builtin_amdgcn_readlane((int)cc, h);
    n.g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cg), h));
    n.vmin = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cvm), h));
    n.x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cx), h));
    n.y = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cy), h));
    n.h = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ch), h));
    n.prev = __builtin_amdgcn_readlane(cpv, h);
    return n;
  }
  __device__ __forceinline__ void sL(int x, int v) {
    t[x].l = v;
    cl = cid == x ? v : cl;
  }
  __device__ __forceinline__ void sR(int x, int v) {
    t[x].r = v;
    cr = cid == x ? v : cr;
  }
  __device__ __forceinline__ void sP(int x, int v) {
    t[x].p = v;
    cp = cid == x ? v : cp;
  }
  __device__ __forceinline__ void sC(int x, int v) {
    *(__attribute__((address_space(1))) uint8_t*)&t[x].cc = (uint8_t)v;  // byte 0 only: ci stays
    cc = cid == x ? ((cc & ~0xffu) | (uint32_t)(v & 0xff)) : cc;
  }
  // the walk step at `depth`: node x, kept in path lane `depth` (copied there on a hit
  // in another lane)
  __device__ __forceinline__ Quad quad_at(int x, int depth) {
    const int h = hit(x);
#ifdef HASTAR_STAMPS
    n_step++;
#endif
    Quad q;
    if (h >= 0) {
      q.key = (uint32_t)__builtin_amdgcn_readlane((int)ck, h);
      q.f = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), h));
      q.l = __builtin_amdgcn_readlane(cl, h);
      q.r = __builtin_amdgcn_readlane(cr, h);
      if (depth < PATH && h != depth) copy_from(x, h, depth);
      return q;
    }
    const Node3 n = fill(x, depth < PATH ? depth : victim(x));
    q.key = n.key;
    q.f = n.f;
    q.l = n.l;
    q.r = n.r;
    return q;
  }

  // The walks of std::set::find (ins = false: go left iff !(node < probe), remember the
  // last node where it went left) and _M_get_insert_unique_pos (ins = true: go left iff
  // probe < node, remember the last node and the last decision), comparator
  // (ka != kb) && (fa < fb).  Outputs as RBT::find / RBT::insert_pos expect them.
  // For insert walks, *rj_ / *rk_ / *rf_ = the deepest node where the walk turned right
  // (rj = -1 if it never did).
  __device__ __forceinline__ void path_walk(uint32_t k, float f, bool ins, int* y_, uint32_t* yk_, float* yf_,
                                            bool* comp_, int* rj_, uint32_t* rk_, float* rf_) {
#ifdef HASTAR_STAMPS
    const unsigned long long tw0 = __builtin_amdgcn_s_memtime();
#endif
    int y = 0, depth = 0;
    uint32_t yk = 0;
    float yf = 0.0f;
    bool comp = true;
    int rj = -1;
    uint32_t rk = 0;
    float rf = 0.0f;
    int x = P(0);
    if (x != NIL && plen > 0 && __builtin_amdgcn_readlane(cid, 0) == x) {
      const bool inpath = lane < plen;
      const bool left = ins ? rb_less(k, f, ck, cf) : !rb_less(ck, cf, k, f);
      const int child = left ? cl : cr;
      const int nxt = __shfl_down(cid, 1, 64);
      const bool cont = inpath && lane + 1 < plen && child == nxt;
      const uint64_t stop = __ballot(!cont);
      const int D = (int)__ffsll((unsigned long long)stop) - 1;  // node D is on the path; leave it via child
      const uint64_t lmask = __ballot(inpath && left) & (D >= 63 ? ~0ull : ((2ull << D) - 1));
      if (ins) {
        y = __builtin_amdgcn_readlane(cid, D);
        yk = (uint32_t)__builtin_amdgcn_readlane((int)ck, D);
        yf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), D));
        comp = (lmask >> D) & 1ull;
        const uint64_t rmask = __ballot(inpath && !left) & (D >= 63 ? ~0ull : ((2ull << D) - 1));
        if (rmask) {
          const int h = 63 - __builtin_clzll(rmask);
          rj = __builtin_amdgcn_readlane(cid, h);
          rk = (uint32_t)__builtin_amdgcn_readlane((int)ck, h);
          rf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), h));
        }
      } else if (lmask) {
        const int h = 63 - __builtin_clzll(lmask);
        y = __builtin_amdgcn_readlane(cid, h);
        yk = (uint32_t)__builtin_amdgcn_readlane((int)ck, h);
        yf = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cf), h));
      }
      x = __builtin_amdgcn_readlane(child, D);
      depth = D + 1;
    }
    while (x != NIL) {
      const Quad q = quad_at(x, depth++);
      if (ins) {
        y = x;
        yk = q.key;
        yf = q.f;
        comp = rb_less(k, f, q.key, q.f);
        if (!comp) {
          rj = y;
          rk = yk;
          rf = yf;
        }
        x = comp ? q.l : q.r;
      } else if (!rb_less(q.key, q.f, k, f)) {
        y = x;
        yk = q.key;
        yf = q.f;
        x = q.l;
      } else {
        x = q.r;
      }
    }
    plen = depth < PATH ? depth : PATH;
#ifdef HASTAR_STAMPS
    pw_cyc += __builtin_amdgcn_s_memtime() - tw0;
    if (ins) pw_ins_cyc += __builtin_amdgcn_s_memtime() - tw0;
#endif
    *y_ = y;
    *yk_ = yk;
    *yf_ = yf;
    *comp_ = comp;
    *rj_ = rj;
    *rk_ = rk;
    *rf_ = rf;
  }
  // a node just written in full by the caller (pool allocation): drop stale copies of
  // the index and cache the new contents (no HBM traffic)
  __device__ __forceinline__ void fresh(int x, const Node3& n) {
    cid = cid == x ? -1 : cid;
    const int slot = victim(x);
    if (lane == slot) set_lane(x, n);
  }
  // RBT::link's first step: the caller has already stored the leaf fields with the node
  __device__ __forceinline__ void leaf(int, int) {}
};
#endif

// Pool allocator for tree nodes: bump pointer + intrusive free list through .l.
struct PoolState {
  int next;   // next never-used index (index 0 is the header)
  int free;   // head of the free list (NIL if empty)
};

// pool over any tree layout (free list through the left link)
template <class Acc>
RB_HD int tpool_alloc(Acc& a, PoolState& ps, int cap) {
  if (ps.free != NIL) {
    const int i = ps.free;
    ps.free = a.L(i);
    return i;
  }
  if (ps.next >= cap) return NIL;
  return ps.next++;
}
template <class Acc>
RB_HD void tpool_free(Acc& a, PoolState& ps, int i) {
  a.sL(i, ps.free);
  ps.free = i;
}

template <class PtrT>
RB_HD int pool_alloc(PtrT t, PoolState& ps, int cap) {
  if (ps.free != NIL) {
    const int i = ps.free;
    ps.free = t[i].l;
    return i;
  }
  if (ps.next >= cap) return NIL;
  return ps.next++;
}

template <class PtrT>
RB_HD void pool_free(PtrT t, PoolState& ps, int i) {
  t[i].l = ps.free;
  ps.free = i;
}

}  // namespace hastar
