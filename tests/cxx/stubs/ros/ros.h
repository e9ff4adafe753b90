// Minimal stand-in for the ROS 1 client API that src/local_planner.cpp uses (TEST HARNESS ONLY:
// tests/test_local_planner.py compiles the reference's unchanged local_planner.cpp against the
// drop-in planner headers with these stubs; no ROS is installed in this image).
//
// Functional, not just declarations: parameters come from an in-process table, subscribe()
// registers the callback under its topic, spinOnce() delivers queued messages, publish()
// keeps the last message per topic, and ros::ok() stays true for a set number of loop turns,
// so a test driver can run the node's own run() loop against a scripted scenario.
#pragma once
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <iterator>
#include <limits>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <type_traits>
#include <vector>

namespace ros {
namespace stub {
// parameter server: string -> value text (numbers) or vector
struct Params {
  std::map<std::string, double> num;
  std::map<std::string, std::vector<double>> vec;
  std::map<std::string, std::string> str;
};
inline Params& params() {
  static Params p;
  return p;
}
// subscriptions: topic -> callback taking a type-erased message
inline std::map<std::string, std::vector<std::function<void(const std::shared_ptr<const void>&)>>>& subs() {
  static std::map<std::string, std::vector<std::function<void(const std::shared_ptr<const void>&)>>> s;
  return s;
}
inline std::vector<std::pair<std::string, std::shared_ptr<const void>>>& queue() {
  static std::vector<std::pair<std::string, std::shared_ptr<const void>>> q;
  return q;
}
inline std::map<std::string, std::shared_ptr<const void>>& published() {
  static std::map<std::string, std::shared_ptr<const void>> p;
  return p;
}
inline int& ok_turns() {
  static int n = 0;
  return n;
}
template <class M>
void deliver(const std::string& topic, const M& msg) {
  queue().emplace_back(topic, std::make_shared<const M>(msg));
}
template <class M>
const M* last(const std::string& topic) {
  auto it = published().find(topic);
  return it == published().end() ? nullptr : static_cast<const M*>(it->second.get());
}
}  // namespace stub

inline void init(int&, char**, const std::string&) {}
inline bool ok() { return stub::ok_turns()-- > 0; }
inline void spinOnce() {
  auto q = std::move(stub::queue());
  stub::queue().clear();
  for (auto& m : q)
    for (auto& cb : stub::subs()[m.first]) cb(m.second);
}

class Rate {
 public:
  template <class T>
  explicit Rate(T) {}
  void sleep() {}
};

class Subscriber {};

class Publisher {
 public:
  std::string topic;
  template <class M>
  void publish(const M& msg) const {
    stub::published()[topic] = std::make_shared<const M>(msg);
  }
};

class NodeHandle {
 public:
  template <class T, class D>
  bool param(const std::string& name, T& out, const D& def) const {
    if constexpr (std::is_same<T, std::string>::value) {
      auto it = stub::params().str.find(name);
      out = it == stub::params().str.end() ? T(def) : it->second;
      return it != stub::params().str.end();
    } else {
      auto it = stub::params().num.find(name);
      out = it == stub::params().num.end() ? static_cast<T>(def) : static_cast<T>(it->second);
      return it != stub::params().num.end();
    }
  }
  template <class T>
  bool getParam(const std::string& name, std::vector<T>& out) const {
    auto it = stub::params().vec.find(name);
    if (it == stub::params().vec.end()) return false;
    out.assign(it->second.begin(), it->second.end());
    return true;
  }
  template <class M, class C>
  Subscriber subscribe(const std::string& topic, uint32_t, void (C::*fp)(const std::shared_ptr<const M>&), C* obj) {
    stub::subs()[topic].push_back([fp, obj](const std::shared_ptr<const void>& m) {
      (obj->*fp)(std::static_pointer_cast<const M>(m));
    });
    return Subscriber();
  }
  template <class M>
  Publisher advertise(const std::string& topic, uint32_t, bool = false) {
    Publisher p;
    p.topic = topic;
    return p;
  }
};
}  // namespace ros

#define ROS_INFO(...)                 \
  do {                                \
    std::fprintf(stderr, __VA_ARGS__); \
    std::fputc('\n', stderr);         \
  } while (0)
#define ROS_INFO_STREAM(x)                      \
  do {                                          \
    std::ostringstream os_;                     \
    os_ << x;                                   \
    std::fprintf(stderr, "%s", os_.str().c_str()); \
  } while (0)
