// rbtree_defer_check.cpp — the deferred inner tree (hastar_kernels.hip, Pend / pend_replay),
// checked on the host: one tree takes every operation at once (insert at the position
// _M_get_insert_unique_pos walks to, erase of the leftmost or of any node), the other only
// logs them — {node, insert flag, in-order predecessor, in-order successor at the insert} —
// and replays the log at random points with the kernel's rule (the right child of the
// predecessor when that slot is free, else the left child of the successor; into the empty
// tree under the header).  After every replay both trees must have the same links, parents,
// colours and header, node for node.  Freed nodes go to a LIFO list kept outside the links
// (the kernel keeps it in the dead nodes' f), so a node whose erase is still in the log keeps
// its links until the replay unlinks it; freed indices are reused while their erase is pending.
//   g++ -O2 -std=c++17 -I path_planning_pkg_amd/csrc tools/rbtree_defer_check.cpp -o /tmp/rbtree_defer_check
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "rbtree_dev.h"

using namespace hastar;

struct Entry {
  int x;
  bool ins;
  int pred, at;
};

int main(int argc, char** argv) {
  const int streams = argc > 1 ? atoi(argv[1]) : 200;
  const int ops = argc > 2 ? atoi(argv[2]) : 20000;
  long long replays = 0, replayed = 0, compared = 0;
  for (int s = 0; s < streams; ++s) {
    std::mt19937_64 rng(777 + s);
    const int cap = 64 + (int)(rng() % 2000);
    std::vector<Node2> pa(cap + 1), pb(cap + 1);
    RBTree<Node2> direct{{pa.data()}}, deferred{{pb.data()}};
    direct.clear();
    deferred.clear();
    std::vector<int> freel;            // LIFO free list (outside the links)
    std::vector<char> live(cap + 1, 0);
    int next = 1, n_live = 0;
    std::vector<Entry> log;
    const int every = 1 + (int)(rng() % 300);  // mean operations between replays
    auto replay = [&]() {
      for (const Entry& e : log) {
        if (!e.ins) {
          deferred.unlink(e.x);
          continue;
        }
        int parent;
        bool left;
        if (e.pred == NIL && e.at == NIL) {
          parent = 0;
          left = true;
        } else if (e.pred == NIL) {
          parent = e.at;
          left = true;
        } else if (e.at == NIL || deferred.R(e.pred) == NIL) {
          parent = e.pred;
          left = false;
        } else {
          parent = e.at;
          left = true;
        }
        pb[e.x].key = pa[e.x].key;  // (the payload the kernel writes at the insert)
        pb[e.x].f = pa[e.x].f;
        deferred.link(left, e.x, parent);
      }
      replayed += (long long)log.size();
      log.clear();
      ++replays;
      for (int i = 0; i < next; ++i) {
        if (i != 0 && !live[i]) continue;
        ++compared;
        if (pa[i].l != pb[i].l || pa[i].r != pb[i].r || pa[i].p != pb[i].p || pa[i].color != pb[i].color) {
          printf("tree mismatch s=%d node=%d\n", s, i);
          return false;
        }
      }
      return true;
    };
    for (int op = 0; op < ops; ++op) {
      const int kind = (int)(rng() % 10);
      if (kind < 3 && n_live > 0) {  // pop the leftmost
        const int b = direct.begin();
        direct.unlink(b);
        live[b] = 0;
        --n_live;
        freel.push_back(b);
        log.push_back({b, false, NIL, NIL});
      } else if (kind < 4 && n_live > 0) {  // erase some live node (a replaced find hit)
        int x;
        do x = 1 + (int)(rng() % (next - 1)); while (!live[x]);
        direct.unlink(x);
        live[x] = 0;
        --n_live;
        freel.push_back(x);
        log.push_back({x, false, NIL, NIL});
      } else if (n_live < cap - 1) {  // insert a node with a unique f (the consistent case)
        int n;
        if (!freel.empty()) {
          n = freel.back();
          freel.pop_back();
        } else if (next <= cap) {
          n = next++;
        } else {
          continue;
        }
        const float f = (float)(rng() % 1000000007ull) * 0.25f + (float)op * 1e-3f;
        const uint32_t key = (uint32_t)(op + 1);
        bool left;
        const int p = direct.insert_pos(key, f, &left);
        if (p == -2) {  // an equal f: dropped (no node)
          freel.push_back(n);
          continue;
        }
        pa[n].key = key;
        pa[n].f = f;
        direct.link(left, n, p);
        live[n] = 1;
        ++n_live;
        // its in-order neighbours now = the rank neighbours the ring gives the kernel
        int pred = NIL, at = NIL;
        {
          int y = n;
          if (direct.L(y) != NIL) {
            y = direct.L(y);
            while (direct.R(y) != NIL) y = direct.R(y);
            pred = y;
          } else {
            int q = direct.P(y);
            while (q != 0 && y == direct.L(q)) { y = q; q = direct.P(q); }
            pred = q == 0 ? NIL : q;
          }
          y = n;
          if (direct.R(y) != NIL) {
            y = direct.R(y);
            while (direct.L(y) != NIL) y = direct.L(y);
            at = y;
          } else {
            int q = direct.P(y);
            while (q != 0 && y == direct.R(q)) { y = q; q = direct.P(q); }
            at = q == 0 ? NIL : q;
          }
        }
        log.push_back({n, true, pred, at});
      }
      if ((int)(rng() % every) == 0 && !replay()) return 1;
    }
    if (!replay()) return 1;
  }
  printf("OK replays=%lld entries=%lld nodes_compared=%lld\n", replays, replayed, compared);
  return 0;
}
