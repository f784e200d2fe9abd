// fifo_arena.h — the host overflow's fixed-capacity FIFO allocator (espgpu.cpp
// Overflow), in a header of its own so the CPU self-test
// (tools/fifo_selftest.cpp) checks the same code against a reference deque.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <new>
#include <type_traits>

namespace espgpu {

// A fixed-capacity FIFO of variable-length contiguous allocations (a bip
// buffer): allocated in arrival order, freed oldest first, wrapping to the
// start when the end has no room.  Allocated once; never grows or moves, so
// process() never reallocates or copies it.
template <class T>
struct FifoArena {
  std::unique_ptr<T[]> buf;
  size_t cap = 0, head = 0, tail = 0;
  bool wrapped = false;              // the newest allocations sit in [0, tail) below head
  size_t wrap_end = 0;               // wrapped: the end of the older region [head, wrap_end)
  // Reserve n elements; false (and the arena unchanged) if that fails.
  bool init(size_t n) {
    T *p = nullptr;
    if (n) {
      p = new (std::nothrow) T[n];
      if (!p) return false;
      if constexpr (std::is_trivially_default_constructible<T>::value) {
        // commit the pages now, one write each: process() then takes no
        // first-touch page fault inside its non-blocking bound
        volatile uint8_t *b = reinterpret_cast<volatile uint8_t *>(p);
        for (size_t o = 0; o < n * sizeof(T); o += 4096) b[o] = 0;
      }
    }
    buf.reset(p);
    cap = n;
    clear();
    return true;
  }
  void swap(FifoArena &o) {
    buf.swap(o.buf);
    std::swap(cap, o.cap);
    std::swap(head, o.head);
    std::swap(tail, o.tail);
    std::swap(wrapped, o.wrapped);
    std::swap(wrap_end, o.wrap_end);
  }
  void clear() { head = tail = wrap_end = 0; wrapped = false; }
  bool empty() const { return !wrapped && head == tail; }
  struct Mark { size_t head, tail, wrap_end; bool wrapped; };
  Mark mark() const { return {head, tail, wrap_end, wrapped}; }
  void undo(const Mark &m) { head = m.head; tail = m.tail; wrap_end = m.wrap_end; wrapped = m.wrapped; }
  // offset of n contiguous elements, or SIZE_MAX when there is no room
  size_t alloc(size_t n) {
    if (n == 0) return 0;
    if (empty()) clear();            // an empty arena restarts at 0: all of cap is contiguous again
    if (!wrapped) {
      if (tail + n <= cap) { tail += n; return tail - n; }
      if (n <= head) { wrapped = true; wrap_end = tail; tail = n; return 0; }
      return SIZE_MAX;
    }
    if (tail + n <= head) { tail += n; return tail - n; }
    return SIZE_MAX;
  }
  // free the oldest allocation [off, off + n)
  void pop(size_t off, size_t n) {
    if (n == 0) return;
    head = off + n;
    if (wrapped && head == wrap_end) {
      // the older region is gone: the oldest allocation left starts at 0
      wrapped = false;
      head = 0;
    }
    if (empty()) clear();
  }
};

}  // namespace espgpu
