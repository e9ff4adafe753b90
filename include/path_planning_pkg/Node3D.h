// Node3D.h — search node of Hybrid A* (reference include/path_planning_pkg/Node3D.h:17-99,
// lib/Node3D.cpp:6-62), a host value type.  The reference's semantics are kept on purpose:
// operator== compares the base cell only (Node3D.h:42 tests `left._angle_bin ==
// left._angle_bin`), operator!= compares cell and heading bin, ordering is (!= and f <),
// set_accumulated_cost ADDS g to f, set_heuristic_cost adds max(h, base node f).
// Nodes without a base node compare by angle bin alone.
#ifndef NODE3D
#define NODE3D

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <iostream>

#include "Node2D.h"
#include "common.h"

namespace planning {

template <typename T>
struct Node3D {
  Vector3D<T> _pose2D;          // pose
  T _cost_g;                    // cost from the start
  T _cost_f;                    // g + heuristic
  T _vmin_sqr;                  // squared minimum arrival speed
  int _curvature_index;         // action that reached this node
  int _angle_bin;               // discrete heading
  const Node2D<T>* _base_node;  // the grid node of this node's cell
  const Node3D<T>* _prev;       // predecessor

  Node3D(Vector3D<T>& pose2D, T cost_g, T vmin_sqr, int curvature_index, int angle_bin, const Node2D<T>* base_node,
         const Node3D<T>* prev)
      : _pose2D(pose2D), _cost_g(cost_g), _cost_f(cost_g), _vmin_sqr(vmin_sqr), _curvature_index(curvature_index),
        _angle_bin(angle_bin), _base_node(base_node), _prev(prev) {}
  Node3D(Vector3D<T>& pose2D, T cost_g, T vmin_sqr, int curvature_index, int angle_bin, const Node3D<T>* prev)
      : Node3D(pose2D, cost_g, vmin_sqr, curvature_index, angle_bin, nullptr, prev) {}
  Node3D() : _cost_g(T(0)), _cost_f(T(0)), _vmin_sqr(T(0)), _curvature_index(0), _angle_bin(0), _base_node(nullptr),
             _prev(nullptr) {}

  void set_accumulated_cost(const T cost_g) {
    _cost_g = cost_g;
    _cost_f += cost_g;
  }
  void set_heuristic_cost(const T cost_h) { _cost_f += _base_node ? std::max(cost_h, _base_node->_cost_f) : cost_h; }
  void soft_reset() {
    _cost_g = T(0);
    _cost_f = T(0);
    _prev = nullptr;
  }

  static bool same_cell(const Node3D& a, const Node3D& b) {
    if (a._base_node && b._base_node) return *a._base_node == *b._base_node;
    return a._base_node == b._base_node;
  }
  friend bool operator==(const Node3D& a, const Node3D& b) { return same_cell(a, b); }
  friend bool operator!=(const Node3D& a, const Node3D& b) { return !same_cell(a, b) || a._angle_bin != b._angle_bin; }
  friend bool operator<(const Node3D& a, const Node3D& b) { return a != b && a._cost_f < b._cost_f; }
  friend bool operator<=(const Node3D& a, const Node3D& b) { return a != b && a._cost_f <= b._cost_f; }
  friend bool operator>(const Node3D& a, const Node3D& b) { return a != b && a._cost_f > b._cost_f; }
  friend bool operator>=(const Node3D& a, const Node3D& b) { return a != b && a._cost_f >= b._cost_f; }
  friend std::ostream& operator<<(std::ostream& os, const Node3D& n) {
    if (n._base_node) os << "xd = " << n._base_node->_posd._x << " yd = " << n._base_node->_posd._y << "\n";
    os << "x = " << n._pose2D._x << " y = " << n._pose2D._y << " heading = " << n._pose2D._heading << "\n"
       << "cost_g = " << n._cost_g << " cost_h = " << (n._cost_f - n._cost_g) << " cost_f = " << n._cost_f << "\n"
       << "vmin_sqr = " << n._vmin_sqr << " curvature_index = " << n._curvature_index
       << " angle_bin = " << n._angle_bin << "\n" << std::endl;
    return os;
  }
  struct HashFunction {
    size_t operator()(const Node3D& n) const {
      const int x = n._base_node ? n._base_node->_posd._x : 0, y = n._base_node ? n._base_node->_posd._y : 0;
      uint64_t z = ((uint64_t)(uint32_t)x << 40) ^ ((uint64_t)(uint32_t)y << 16) ^ (uint32_t)n._angle_bin;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      return (size_t)(z ^ (z >> 31));
    }
  };
};

}  // namespace planning

#endif  // NODE3D
