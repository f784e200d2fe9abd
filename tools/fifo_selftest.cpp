// CPU self-test of the host overflow's allocator (f-stack_amd/csrc/fifo_arena.h,
// espgpu.cpp Overflow): random alloc / pop sequences, with wraps, undos of
// partial allocations and an empty arena that restarts at 0, checked against a
// reference model -- every live allocation lies inside the arena, no two
// overlap, pops come back oldest first, and an allocation is refused only when
// no contiguous free run of that size exists where a bip buffer may place it.
// Run by tests/test_host_selftests.py.
#include <stdio.h>
#include <stdlib.h>

#include <deque>
#include <random>

#include "fifo_arena.h"

using espgpu::FifoArena;

namespace {

struct Live { size_t off, n; };

int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      printf("FAIL line %d: %s\n", __LINE__, #c);                  \
      if (++fails > 20) exit(1);                                   \
    }                                                              \
  } while (0)

// Whether a bip buffer holding exactly the live allocations q (oldest first)
// must place n more: after the newest if it fits before the end (one region)
// or before the oldest (wrapped: the newest region starts at 0 below the
// oldest), or at 0 when one region leaves n free before it; an empty arena
// takes any n <= cap.
bool model_fits(const std::deque<Live> &q, size_t cap, size_t n) {
  if (n == 0) return true;
  if (q.empty()) return n <= cap;
  const size_t head = q.front().off, tail = q.back().off + q.back().n;
  const bool wrapped = q.back().off < head;      // the newest lies below the oldest
  if (!wrapped) return tail + n <= cap || n <= head;
  return tail + n <= head;
}

void run(size_t cap, uint32_t seed, int steps) {
  FifoArena<uint8_t> a;
  CHECK(a.init(cap));
  std::deque<Live> q;
  std::mt19937 rng(seed);
  for (int s = 0; s < steps; ++s) {
    const uint32_t r = rng() % 100;
    if (r < 55) {
      const size_t n = rng() % 4 == 0 ? rng() % (cap + 2) : 1 + rng() % (cap / 8 + 1);
      const bool fits = model_fits(q, cap, n);
      const auto m = a.mark();
      const size_t off = a.alloc(n);
      if (rng() % 8 == 0 && off != SIZE_MAX) {
        a.undo(m);                               // a partial placement rolled back (process())
        continue;
      }
      CHECK((off != SIZE_MAX) == fits);
      if (off == SIZE_MAX || n == 0) continue;
      CHECK(off + n <= cap);
      for (const Live &l : q) CHECK(off + n <= l.off || l.off + l.n <= off);
      q.push_back({off, n});
    } else if (!q.empty()) {
      const Live l = q.front();
      q.pop_front();
      a.pop(l.off, l.n);
      if (q.empty()) {
        CHECK(a.empty());
        CHECK(a.alloc(cap) == 0);                // an empty arena is whole again
        a.pop(0, cap);
      }
    }
  }
  while (!q.empty()) {
    a.pop(q.front().off, q.front().n);
    q.pop_front();
  }
  CHECK(a.empty());
}

}  // namespace

int main() {
  for (uint32_t seed = 1; seed <= 200; ++seed) run(64 + seed * 37 % 4096, seed, 4000);
  run(1, 7, 1000);
  run(4, 9, 1000);
  if (fails) return 1;
  printf("OK fifo arena\n");
  return 0;
}
