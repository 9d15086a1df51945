// Host sanitizer driver for the DDP bucket planner / ready tracker core (csrc/ddp_reducer_core.h), SURVEY §5.2:
// randomised parameter lists (tiny and oversized parameters, one or two optimizer regions, a tied weight, world
// sizes 1-8, split on / off) through plan() and Tracker, checking the layout invariants the engine relies on:
//   * parameters are disjoint, align-rounded slices of [0, numel) in the given order;
//   * buckets are consecutive, pad-unit-aligned, non-empty, ordered, and cover every parameter slice they own;
//   * a split parameter's owner buckets are consecutive; a tied weight's buckets hold only it (replicated);
//   * the tracker launches every bucket exactly once, in index order, only after all its parameters are marked,
//     and rejects a second signal of one parameter in one backward.
// Built and run by tests/test_sanitizers_cpu.py:
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -I csrc reducer_sanitize.cpp
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "ddp_reducer_core.h"

using namespace sftamd::reducer;

#define CHECK(c)                                                                \
  do {                                                                          \
    if (!(c)) {                                                                 \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  std::mt19937_64 rng(4321);
  const int64_t size_menu[] = {3, 1, 7, 64, 1000, 4096, 70000, 300000, 2000000};
  for (int it = 0; it < iters; ++it) {
    const int64_t np = 1 + rng() % 50;
    std::vector<int64_t> sizes(np), region(np);
    const int64_t nd = rng() % (np + 1);
    for (int64_t i = 0; i < np; ++i) {
      sizes[i] = size_menu[rng() % 9];
      region[i] = i < nd ? 0 : 1;
    }
    const int64_t world = 1 << (rng() % 4);
    const int64_t align = 64, pad_unit = 2048 * world;
    const int64_t caps[] = {pad_unit, 50000, 400000};
    const int64_t cap = std::max(pad_unit, caps[rng() % 3]);
    const int64_t first_cap = std::max(pad_unit, (int64_t)(rng() % 2 ? 20000 : 1));
    const int64_t split_at = rng() % 2 ? 2 * cap : 0;
    const int64_t tied = rng() % 2 ? -1 : 0;  // the engine puts the tied weight first in the layout
    const std::vector<int64_t> p = plan(sizes, region, tied, align, pad_unit, cap, first_cap, split_at);
    // unpack (bounds-checked: the vector is exactly sized)
    CHECK(p.size() >= 5);
    const int64_t numel = p[0], nb = p[1], n = p[2], nr = p[3];
    CHECK(n == np && nb >= 1 && nr >= 1 && nr <= 2);
    size_t k = 4;
    auto take = [&](int64_t cnt) {
      CHECK(k + (size_t)cnt <= p.size());
      std::vector<int64_t> v(p.begin() + k, p.begin() + k + cnt);
      k += cnt;
      return v;
    };
    const auto off = take(np), bs = take(nb), be = take(nb), br = take(nb), ptr = take(np + 1);
    const auto own = take(ptr.back());
    const auto regs = take(3 * nr);
    take(1);
    CHECK(k == p.size());
    // parameters: ordered, disjoint, aligned
    for (int64_t i = 0; i < np; ++i) {
      CHECK(off[i] % align == 0 && off[i] >= 0 && off[i] + sizes[i] <= numel);
      if (i) CHECK(off[i] >= off[i - 1] + rup(sizes[i - 1], align));
    }
    // buckets: ordered, aligned, non-empty
    std::vector<int> nparams(nb, 0);
    for (int64_t b = 0; b < nb; ++b) {
      CHECK(bs[b] % pad_unit == 0 && be[b] % pad_unit == 0 && be[b] > bs[b] && be[b] <= numel);
      if (b) CHECK(bs[b] >= be[b - 1]);
    }
    for (int64_t i = 0; i < np; ++i) {
      CHECK(ptr[i + 1] > ptr[i]);
      for (int64_t q = ptr[i]; q < ptr[i + 1]; ++q) {
        CHECK(own[q] >= 0 && own[q] < nb);
        if (q > ptr[i]) CHECK(own[q] == own[q - 1] + 1);
        ++nparams[own[q]];
      }
      // the owner buckets cover the parameter's slice
      CHECK(bs[own[ptr[i]]] <= off[i] && be[own[ptr[i + 1] - 1]] >= off[i] + sizes[i]);
      if (i == tied)
        for (int64_t q = ptr[i]; q < ptr[i + 1]; ++q) CHECK(br[own[q]] == 1);
    }
    for (int64_t b = 0; b < nb; ++b) {
      CHECK(nparams[b] >= 1);
      if (br[b]) CHECK(nparams[b] == 1);
    }
    for (int64_t r = 0; r < nr; ++r) CHECK(regs[3 * r] <= regs[3 * r + 1] && regs[3 * r + 1] <= numel);
    // tracker: random mark orders over two backwards
    Tracker t(ptr, own, nb);
    for (int pass = 0; pass < 2; ++pass) {
      t.reset();
      std::vector<int64_t> order(np);
      for (int64_t i = 0; i < np; ++i) order[i] = i;
      std::shuffle(order.begin(), order.end(), rng);
      const int64_t cut = rng() % (np + 1);
      std::vector<int> launched(nb, 0), left(nparams.begin(), nparams.end());
      int64_t expect_next = 0;
      for (int64_t j = 0; j < cut; ++j) {
        const int64_t i = order[j];
        for (int64_t q = ptr[i]; q < ptr[i + 1]; ++q) --left[own[q]];
        for (int64_t b : t.mark(i)) {
          CHECK(b == expect_next++ && left[b] == 0 && !launched[b]);
          launched[b] = 1;
        }
      }
      for (int64_t b : t.drain()) {
        CHECK(b == expect_next++ && !launched[b]);
        launched[b] = 1;
      }
      CHECK(expect_next == nb);
      if (cut > 0) {
        bool threw = false;
        try {
          t.mark(order[0]);
        } catch (const std::runtime_error&) {
          threw = true;
        }
        CHECK(threw);
      }
    }
  }
  std::printf("reducer core clean after %d plans\n", iters);
  return 0;
}
