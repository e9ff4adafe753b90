// Node2D.h — grid node of the holonomic heuristic search (reference
// include/path_planning_pkg/Node2D.h:15-84, lib/Node2D.cpp:6-40), a host value type.
// Equality is by cell; ordering is the reference's (cells differ AND f compares), which is
// not a strict weak order: std::set<Node2D> built from it drops equal-f inserts exactly as
// the reference's open sets do.  The hash mixes the cell with a 64-bit finaliser instead of
// boost::hash_combine (set semantics are hash-independent; no Boost dependency).
#ifndef NODE2D
#define NODE2D

#include <cstddef>
#include <cstdint>
#include <iostream>

#include "common.h"

namespace planning {

template <typename T>
struct Node2D {
  Vector2D<int> _posd;     // cell indices
  T _cost_g;               // cost from the start
  T _cost_h;               // heuristic to the goal
  T _cost_f;               // g + h
  const Node2D<T>* _prev;  // predecessor

  Node2D(int xd, int yd, T cost_g, T cost_h, const Node2D<T>* prev)
      : _posd(xd, yd), _cost_g(cost_g), _cost_h(cost_h), _cost_f(cost_g + cost_h), _prev(prev) {}
  Node2D(int xd, int yd) : Node2D(xd, yd, T(0), T(0), nullptr) {}

  void set_accumulated_cost(const T cost_g) {
    _cost_g = cost_g;
    _cost_f = cost_g + _cost_h;
  }
  void set_heuristic_cost(const T cost_h) {
    _cost_h = cost_h;
    _cost_f = _cost_g + cost_h;
  }
  void soft_reset() {  // keeps the cell and h
    _cost_g = T(0);
    _cost_f = _cost_h;
    _prev = nullptr;
  }

  friend bool operator==(const Node2D& a, const Node2D& b) { return a._posd._x == b._posd._x && a._posd._y == b._posd._y; }
  friend bool operator!=(const Node2D& a, const Node2D& b) { return !(a == b); }
  friend bool operator<(const Node2D& a, const Node2D& b) { return a != b && a._cost_f < b._cost_f; }
  friend bool operator<=(const Node2D& a, const Node2D& b) { return a != b && a._cost_f <= b._cost_f; }
  friend bool operator>(const Node2D& a, const Node2D& b) { return a != b && a._cost_f > b._cost_f; }
  friend bool operator>=(const Node2D& a, const Node2D& b) { return a != b && a._cost_f >= b._cost_f; }
  friend std::ostream& operator<<(std::ostream& os, const Node2D& n) {
    os << "xd = " << n._posd._x << " yd = " << n._posd._y << "\n"
       << "cost_g = " << n._cost_g << " cost_h = " << n._cost_h << " cost_f = " << n._cost_f << "\n" << std::endl;
    return os;
  }
  struct HashFunction {
    size_t operator()(const Node2D& n) const {
      uint64_t z = ((uint64_t)(uint32_t)n._posd._x << 32) | (uint32_t)n._posd._y;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      return (size_t)(z ^ (z >> 31));
    }
  };
};

}  // namespace planning

#endif  // NODE2D
