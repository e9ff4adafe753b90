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
// Tested against std::set on random operation streams: tests/test_rbtree_host.py.
#pragma once
#include <type_traits>
#include "hastar_layout.h"

#if defined(__HIPCC__)
#define RB_HD __host__ __device__ __forceinline__
#else
#define RB_HD inline
#endif

namespace hastar {

// comparator of the reference: (ka != kb) && (fa < fb)
RB_HD bool rb_less(uint32_t ka, float fa, uint32_t kb, float fb) { return (ka != kb) && (fa < fb); }

// {key, f, l, r} of one node in one 16-byte load (the first 16 bytes of every node type)
struct Quad {
  uint32_t key;
  float f;
  int l, r;
};
#if defined(__HIP_DEVICE_COMPILE__)
typedef int rb_v4i __attribute__((ext_vector_type(4)));
template <class PtrT>
__device__ __forceinline__ Quad rb_quad(PtrT t, int x) {
  typedef typename std::remove_reference<decltype(t[0].key)>::type K;  // keeps the address space
  (void)sizeof(K);
  const rb_v4i v = *reinterpret_cast<decltype(&reinterpret_cast<const rb_v4i&>(t[x]))>(&t[x]);
  Quad q;
  q.key = (uint32_t)v.x;
  q.f = __int_as_float(v.y);
  q.l = v.z;
  q.r = v.w;
  return q;
}
#else
template <class PtrT>
inline Quad rb_quad(PtrT t, int x) {
  return Quad{t[x].key, t[x].f, t[x].l, t[x].r};
}
#endif

template <class NodeT, class PtrT = NodeT*>
struct RBTree {
  PtrT t;

  RB_HD int root() const { return t[0].p; }
  RB_HD int begin() const { return t[0].l; }          // == 0 (header) when empty
  RB_HD bool empty() const { return t[0].p == NIL; }

  RB_HD void clear() {
    t[0].p = NIL;
    t[0].l = 0;
    t[0].r = 0;
    t[0].color = RB_RED;
  }

  RB_HD void rotate_left(int x) {
    const int y = t[x].r;
    t[x].r = t[y].l;
    if (t[y].l != NIL) t[t[y].l].p = x;
    t[y].p = t[x].p;
    if (x == t[0].p) t[0].p = y;
    else if (x == t[t[x].p].l) t[t[x].p].l = y;
    else t[t[x].p].r = y;
    t[y].l = x;
    t[x].p = y;
  }

  RB_HD void rotate_right(int x) {
    const int y = t[x].l;
    t[x].l = t[y].r;
    if (t[y].r != NIL) t[t[y].r].p = x;
    t[y].p = t[x].p;
    if (x == t[0].p) t[0].p = y;
    else if (x == t[t[x].p].r) t[t[x].p].r = y;
    else t[t[x].p].l = y;
    t[y].r = x;
    t[x].p = y;
  }

  RB_HD int decrement(int x) const {
    if (t[x].color == RB_RED && t[x].p != NIL && t[t[x].p].p == x) return t[x].r;  // header
    if (t[x].l != NIL) {
      int y = t[x].l;
      while (t[y].r != NIL) y = t[y].r;
      return y;
    }
    int y = t[x].p;
    while (x == t[y].l) {
      x = y;
      y = t[y].p;
    }
    return y;
  }

  // std::set::find (stl_tree.h _M_lower_bound + key_compare check).  Returns 0 (= end)
  // when not "found".
  RB_HD int find(uint32_t k, float f) const {
    int y = 0, x = t[0].p;
    uint32_t yk = 0;
    float yf = 0.0f;
    while (x != NIL) {
      const Quad q = rb_quad(t, x);
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
  RB_HD int insert_pos(uint32_t k, float f, bool* left) const {
    int x = t[0].p, y = 0;
    bool comp = true;
    while (x != NIL) {
      const Quad q = rb_quad(t, x);
      y = x;
      comp = rb_less(k, f, q.key, q.f);
      x = comp ? q.l : q.r;
    }
    int j = y;
    if (comp) {
      if (j == t[0].l) {
        *left = true;  // _M_insert_: x != 0 is false; p == end() or comp(v, p) holds
        return y;
      }
      j = decrement(j);
    }
    if (rb_less(t[j].key, t[j].f, k, f)) {
      *left = (y == 0) || rb_less(k, f, t[y].key, t[y].f);
      return y;
    }
    return -2;
  }

  // _Rb_tree_insert_and_rebalance(insert_left, x, p, header)
  RB_HD void link(bool insert_left, int x, int p) {
    t[x].p = p;
    t[x].l = NIL;
    t[x].r = NIL;
    t[x].color = RB_RED;
    if (insert_left) {
      t[p].l = x;
      if (p == 0) {
        t[0].p = x;
        t[0].r = x;
      } else if (p == t[0].l) {
        t[0].l = x;
      }
    } else {
      t[p].r = x;
      if (p == t[0].r) t[0].r = x;
    }
    while (x != t[0].p && t[t[x].p].color == RB_RED) {
      const int xp = t[x].p;
      const int xpp = t[xp].p;
      if (xp == t[xpp].l) {
        const int y = t[xpp].r;
        if (y != NIL && t[y].color == RB_RED) {
          t[xp].color = RB_BLACK;
          t[y].color = RB_BLACK;
          t[xpp].color = RB_RED;
          x = xpp;
        } else {
          if (x == t[xp].r) {
            x = xp;
            rotate_left(x);
          }
          t[t[x].p].color = RB_BLACK;
          t[xpp].color = RB_RED;
          rotate_right(xpp);
        }
      } else {
        const int y = t[xpp].l;
        if (y != NIL && t[y].color == RB_RED) {
          t[xp].color = RB_BLACK;
          t[y].color = RB_BLACK;
          t[xpp].color = RB_RED;
          x = xpp;
        } else {
          if (x == t[xp].l) {
            x = xp;
            rotate_right(x);
          }
          t[t[x].p].color = RB_BLACK;
          t[xpp].color = RB_RED;
          rotate_left(xpp);
        }
      }
    }
    t[t[0].p].color = RB_BLACK;
  }

  RB_HD int minimum(int x) const {
    while (t[x].l != NIL) x = t[x].l;
    return x;
  }
  RB_HD int maximum(int x) const {
    while (t[x].r != NIL) x = t[x].r;
    return x;
  }

  // _Rb_tree_rebalance_for_erase(z, header); the caller frees z afterwards.
  RB_HD void unlink(int z) {
    int y = z, x = NIL, xp = NIL;
    if (t[y].l == NIL) {
      x = t[y].r;
    } else if (t[y].r == NIL) {
      x = t[y].l;
    } else {
      y = t[y].r;
      while (t[y].l != NIL) y = t[y].l;
      x = t[y].r;
    }
    if (y != z) {
      t[t[z].l].p = y;
      t[y].l = t[z].l;
      if (y != t[z].r) {
        xp = t[y].p;
        if (x != NIL) t[x].p = t[y].p;
        t[t[y].p].l = x;
        t[y].r = t[z].r;
        t[t[z].r].p = y;
      } else {
        xp = y;
      }
      if (t[0].p == z) t[0].p = y;
      else if (t[t[z].p].l == z) t[t[z].p].l = y;
      else t[t[z].p].r = y;
      t[y].p = t[z].p;
      const int c = t[y].color;
      t[y].color = t[z].color;
      t[z].color = c;
      y = z;
    } else {
      xp = t[y].p;
      if (x != NIL) t[x].p = t[y].p;
      if (t[0].p == z) t[0].p = x;
      else if (t[t[z].p].l == z) t[t[z].p].l = x;
      else t[t[z].p].r = x;
      if (t[0].l == z) t[0].l = (t[z].r == NIL) ? t[z].p : minimum(x);
      if (t[0].r == z) t[0].r = (t[z].l == NIL) ? t[z].p : maximum(x);
    }
    if (t[y].color != RB_RED) {
      while (x != t[0].p && (x == NIL || t[x].color == RB_BLACK)) {
        if (x == t[xp].l) {
          int w = t[xp].r;
          if (t[w].color == RB_RED) {
            t[w].color = RB_BLACK;
            t[xp].color = RB_RED;
            rotate_left(xp);
            w = t[xp].r;
          }
          if ((t[w].l == NIL || t[t[w].l].color == RB_BLACK) && (t[w].r == NIL || t[t[w].r].color == RB_BLACK)) {
            t[w].color = RB_RED;
            x = xp;
            xp = t[xp].p;
          } else {
            if (t[w].r == NIL || t[t[w].r].color == RB_BLACK) {
              t[t[w].l].color = RB_BLACK;
              t[w].color = RB_RED;
              rotate_right(w);
              w = t[xp].r;
            }
            t[w].color = t[xp].color;
            t[xp].color = RB_BLACK;
            if (t[w].r != NIL) t[t[w].r].color = RB_BLACK;
            rotate_left(xp);
            break;
          }
        } else {
          int w = t[xp].l;
          if (t[w].color == RB_RED) {
            t[w].color = RB_BLACK;
            t[xp].color = RB_RED;
            rotate_right(xp);
            w = t[xp].l;
          }
          if ((t[w].r == NIL || t[t[w].r].color == RB_BLACK) && (t[w].l == NIL || t[t[w].l].color == RB_BLACK)) {
            t[w].color = RB_RED;
            x = xp;
            xp = t[xp].p;
          } else {
            if (t[w].l == NIL || t[t[w].l].color == RB_BLACK) {
              t[t[w].r].color = RB_BLACK;
              t[w].color = RB_RED;
              rotate_left(w);
              w = t[xp].l;
            }
            t[w].color = t[xp].color;
            t[xp].color = RB_BLACK;
            if (t[w].l != NIL) t[t[w].l].color = RB_BLACK;
            rotate_right(xp);
            break;
          }
        }
      }
      if (x != NIL) t[x].color = RB_BLACK;
    }
  }
};

// Pool allocator for tree nodes: bump pointer + intrusive free list through .l.
struct PoolState {
  int next;   // next never-used index (index 0 is the header)
  int free;   // head of the free list (NIL if empty)
};

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
