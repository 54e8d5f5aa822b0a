// Compile-time loop helpers shared by the solvers (solver1.hpp,
// solver_mixed.hpp, solver64.hpp, solver64m.hpp).
#pragma once
#include <type_traits>
#include "common.hpp"

namespace danse {

template <int B, int E, typename Fn>
DANSE_DEV void sfor(Fn&& fn) {
  if constexpr (B < E) {
    fn(std::integral_constant<int, B>{});
    sfor<B + 1, E>(fn);
  }
}
// B-1, B-2, ..., E
template <int B, int E, typename Fn>
DANSE_DEV void sfor_down(Fn&& fn) {
  if constexpr (B > E) {
    fn(std::integral_constant<int, B - 1>{});
    sfor_down<B - 1, E>(fn);
  }
}

constexpr int kRMax = 4;   // largest supported GEVD rank

}  // namespace danse
