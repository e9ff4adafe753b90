// rbtree_check.cpp — differential test: rbtree_dev.h vs std::set (libstdc++) with the
// reference's non-strict-weak comparator (Node3D.h:50-54).  Random operation streams
// mimic the planner: pop-min, find-then-insert, find-then-erase+insert, with f values
// drawn from a small set so equal-f collisions (dropped inserts, cross-key finds) are
// frequent.  Exit 0 iff every outcome and every in-order traversal matches.
//   g++ -O2 -std=c++17 -I path_planning_pkg_amd/csrc tools/rbtree_check.cpp -o /tmp/rbtree_check
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>
#include <random>
#include "rbtree_dev.h"

using namespace hastar;

struct E { uint32_t key; float f; int id; };
struct Less { bool operator()(const E& a, const E& b) const { return (a.key != b.key) && (a.f < b.f); } };

int main(int argc, char** argv) {
  const int streams = argc > 1 ? atoi(argv[1]) : 200;
  const int ops = argc > 2 ? atoi(argv[2]) : 20000;
  long long checks = 0, drops = 0, xfinds = 0;
  for (int s = 0; s < streams; ++s) {
    std::mt19937_64 rng(1234 + s);
    const int keyspace = 8 + (int)(rng() % 200);
    const int fspace = 2 + (int)(rng() % 40);
    std::set<E, Less> ref;
    std::vector<Node2> pool(ops + 2);
    RBTree<Node2> tr{{pool.data()}};
    tr.clear();
    PoolState ps{1, NIL};
    std::vector<int> id_of_node(ops + 2, -1);
    int next_id = 0;
    for (int op = 0; op < ops; ++op) {
      int kind = (int)(rng() % 10);
      E e{(uint32_t)(rng() % keyspace), (float)(rng() % fspace) * 0.5f, next_id};
      if (kind < 3 && !ref.empty()) {  // pop-min
        auto it = ref.begin();
        int b = tr.begin();
        if (b == 0 || id_of_node[b] != it->id) { printf("begin mismatch s=%d op=%d\n", s, op); return 1; }
        ref.erase(it);
        tr.unlink(b);
        pool_free(pool.data(), ps, b);
      } else if (kind < 8) {  // find; insert if not found
        auto it = ref.find(e);
        int fnd = tr.find(e.key, e.f);
        bool rf = it != ref.end();
        if (rf != (fnd != 0) || (rf && id_of_node[fnd] != it->id)) { printf("find mismatch s=%d op=%d\n", s, op); return 1; }
        if (rf && it->key != e.key) ++xfinds;
        if (!rf) {
          auto pr = ref.insert(e);
          bool left;
          int p = tr.insert_pos(e.key, e.f, &left);
          if (pr.second != (p != -2)) { printf("insert mismatch s=%d op=%d\n", s, op); return 1; }
          if (p != -2) {
            int n = pool_alloc(pool.data(), ps, (int)pool.size());
            pool[n].key = e.key; pool[n].f = e.f; id_of_node[n] = e.id;
            tr.link(left, n, p);
          } else {
            ++drops;
          }
          ++next_id;
        }
      } else {  // find; if found and "better", erase + reinsert
        auto it = ref.find(e);
        int fnd = tr.find(e.key, e.f);
        bool rf = it != ref.end();
        if (rf != (fnd != 0) || (rf && id_of_node[fnd] != it->id)) { printf("find2 mismatch s=%d op=%d\n", s, op); return 1; }
        if (rf) {
          ref.erase(it);
          tr.unlink(fnd);
          pool_free(pool.data(), ps, fnd);
          E e2{e.key, e.f + 0.25f * (float)(rng() % 3), next_id++};
          auto pr = ref.insert(e2);
          bool left;
          int p = tr.insert_pos(e2.key, e2.f, &left);
          if (pr.second != (p != -2)) { printf("insert2 mismatch s=%d op=%d\n", s, op); return 1; }
          if (p != -2) {
            int n = pool_alloc(pool.data(), ps, (int)pool.size());
            pool[n].key = e2.key; pool[n].f = e2.f; id_of_node[n] = e2.id;
            tr.link(left, n, p);
          }
        }
      }
      // in-order traversal must match element for element
      if (op % 97 == 0 || op == ops - 1) {
        std::vector<int> a, stk;
        for (int x = tr.root(); x != NIL || !stk.empty();) {
          if (x != NIL) { stk.push_back(x); x = pool[x].l; continue; }
          x = stk.back(); stk.pop_back();
          a.push_back(id_of_node[x]);
          x = pool[x].r;
        }
        if ((int)a.size() > ops + 2) { printf("cycle\n"); return 1; }
        std::vector<int> b;
        for (auto& v : ref) b.push_back(v.id);
        if (a != b) { printf("traversal mismatch s=%d op=%d (%zu vs %zu)\n", s, op, a.size(), b.size()); return 1; }
        if (!ref.empty() && pool[tr.begin()].key != ref.begin()->key) { printf("leftmost\n"); return 1; }
        ++checks;
      }
    }
  }
  printf("OK streams=%d ops=%d traversal_checks=%lld dropped_inserts=%lld cross_key_finds=%lld\n", streams, ops,
         checks, drops, xfinds);
  return 0;
}
