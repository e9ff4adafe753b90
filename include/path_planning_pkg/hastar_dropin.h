// hastar_dropin.h — shared plumbing of the drop-in headers in this directory: the HIP
// device they run on ($HASTAR_DEVICE, default 0) and error reporting (a failed device call
// throws std::runtime_error; the reference has no device that could fail).
#ifndef HASTAR_DROPIN_H
#define HASTAR_DROPIN_H

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../hastar_units.h"

namespace planning {
namespace hastar_dropin {
inline int device() {
  const char* d = std::getenv("HASTAR_DEVICE");
  return d ? std::atoi(d) : 0;
}
inline void check(int rc, bool units = false) {
  if (rc < 0)
    throw std::runtime_error(std::string("hastar: ") + (units ? hastar_units_last_error() : hastar_last_error()));
}
}  // namespace hastar_dropin
}  // namespace planning

#endif  // HASTAR_DROPIN_H
