// Host sanitizer driver for the native collator core (csrc/collate_core.h), SURVEY §5.2: randomised corpora
// (empty samples, samples longer than max_length, max_tokens smaller than one sample, pad multiples 1 / 64 / 256)
// through pad_width/pad_fill and pack_plan/pack_fill into EXACTLY-sized heap buffers, so any out-of-bounds write
// or read is an AddressSanitizer error and any signed overflow / bad shift a UBSan error; the outputs are checked
// against a direct reimplementation of the HF semantics. Built and run by tests/test_sanitizers_cpu.py:
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all -I csrc collate_sanitize.cpp
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>

#include "collate_core.h"

using namespace sftamd::collate;

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  std::mt19937_64 rng(1234);
  for (int it = 0; it < iters; ++it) {
    const int64_t nsamp = 1 + rng() % 40;
    std::vector<int64_t> off(nsamp + 1, 0);
    for (int64_t i = 0; i < nsamp; ++i) off[i + 1] = off[i] + (rng() % 5 == 0 ? 0 : (int64_t)(rng() % 700));
    const int64_t ntok = off[nsamp];
    std::unique_ptr<int32_t[]> tok(new int32_t[ntok > 0 ? ntok : 1]);
    for (int64_t t = 0; t < ntok; ++t) tok[t] = (int32_t)(rng() % 128256);
    const int64_t B = 1 + rng() % nsamp;
    std::vector<int64_t> order(B);
    for (auto& o : order) o = rng() % nsamp;
    const int64_t mults[3] = {1, 64, 256};
    const int64_t pm = mults[rng() % 3];
    const int64_t maxlen = rng() % 3 == 0 ? 0 : 1 + (int64_t)(rng() % 1024);

    // ---- padding
    std::vector<int64_t> lens;
    const int64_t T = pad_width(off.data(), order.data(), B, maxlen, pm, lens);
    CHECK(T >= 1 && T % pm == 0);
    std::unique_ptr<int64_t[]> ids(new int64_t[B * T]), lab(new int64_t[B * T]);
    std::unique_ptr<int32_t[]> lengths(new int32_t[B]);
    for (int64_t k = 0; k < B * T; ++k) ids[k] = 7, lab[k] = -100;
    pad_fill(tok.get(), off.data(), order.data(), lens, T, ids.get(), lab.get(), lengths.get());
    for (int64_t b = 0; b < B; ++b) {
      int64_t l = off[order[b] + 1] - off[order[b]];
      if (maxlen > 0 && l > maxlen) l = maxlen;
      CHECK(lengths[b] == l && l <= T);
      for (int64_t t = 0; t < T; ++t) {
        const bool in = t < l;
        CHECK(ids[b * T + t] == (in ? tok[off[order[b]] + t] : 7));
        CHECK(lab[b * T + t] == (in ? tok[off[order[b]] + t] : -100));
      }
    }

    // ---- packing
    const int64_t maxtok = rng() % 4 == 0 ? 0 : 1 + (int64_t)(rng() % 4096);
    std::vector<int64_t> cu;
    const int64_t used = pack_plan(off.data(), order.data(), B, maxtok, cu);
    CHECK(used >= 1 && used <= B && (int64_t)cu.size() == used + 1);
    const int64_t M = cu.back();
    CHECK(maxtok == 0 || M <= maxtok || used == 1);
    const int64_t Mp = round_up(M > 1 ? M : 1, pm);
    const int64_t nseq = used + (Mp > M ? 1 : 0);
    std::unique_ptr<int64_t[]> pid(new int64_t[Mp]), plab(new int64_t[Mp]), pos(new int64_t[Mp]);
    std::unique_ptr<int32_t[]> cus(new int32_t[nseq + 1]);
    for (int64_t k = 0; k < Mp; ++k) pid[k] = 7, plab[k] = -100, pos[k] = 0;
    pack_fill(tok.get(), off.data(), order.data(), cu, Mp, pid.get(), plab.get(), pos.get(), cus.get());
    CHECK(cus[0] == 0 && cus[used] == M && (Mp == M || cus[nseq] == Mp));
    for (int64_t s = 0; s < used; ++s) {
      const int64_t b = cus[s], l = cus[s + 1] - cus[s];
      const int32_t* src = tok.get() + off[order[s]];
      for (int64_t t = 0; t < l; ++t) {
        CHECK(pid[b + t] == src[t] && pos[b + t] == t);
        CHECK(plab[b + t] == (t + 1 < l ? src[t + 1] : -100));
      }
    }
    for (int64_t t = M; t < Mp; ++t) CHECK(pid[t] == 7 && plab[t] == -100 && pos[t] == t - M);
  }
  std::printf("collate_sanitize: %d randomised cases clean\n", iters);
  return 0;
}
