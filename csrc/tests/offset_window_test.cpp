// OffsetWindow (csrc/runtime/engine.h) against a std::set model: random adds / completions with
// seeks back and far forward jumps; the oldest pending offset (the commit position) must always
// agree and the window must stay within its span bound. Built and run by
// tests/test_offset_window.py (host code only).
#include <stdio.h>

#include <random>
#include <set>

#include "../runtime/engine.h"

// A sparse offset that the window later grows over (base stalled, a record set aside past
// kMaxSpan, base moves on, a new add() resizes the window across it) must still complete.
static int sparse_overlap_case() {
  const int64_t S = gale::OffsetWindow::kMaxSpan;
  gale::OffsetWindow w;
  for (int64_t o = 0; o <= 10; ++o) w.add(o);  // offset 0: the stalled record at base
  w.add(S + 5);     // >= kMaxSpan past base: set aside in the sparse set
  for (int64_t o = 0; o < 10; ++o) w.done(o);  // base moves to 10 (still pending)
  w.add(S + 8);     // inside the window now: st grows over S + 5
  w.done(S + 5);    // must leave the sparse set although its window slot is 0
  w.done(10);
  w.done(S + 8);
  if (!w.empty()) {
    fprintf(stderr, "sparse overlap: window not empty (first %lld)\n", (long long)w.first());
    return 1;
  }
  return 0;
}

int main() {
  if (sparse_overlap_case()) return 1;
  std::mt19937_64 rng(42);
  for (int round = 0; round < 200; ++round) {
    gale::OffsetWindow w;
    std::set<int64_t> model;
    int64_t next = (int64_t)(rng() % 1000);
    for (int step = 0; step < 20000; ++step) {
      const int r = (int)(rng() % 100);
      if (r < 55) {  // fetch the next offset
        w.add(next);
        model.insert(next);
        ++next;
      } else if (r < 90 && !model.empty()) {  // complete a random pending one
        auto it = model.begin();
        std::advance(it, (long)(rng() % std::min<size_t>(model.size(), 64)));
        w.done(*it);
        model.erase(it);
      } else if (r < 93) {  // far forward seek (e.g. out-of-range reset to latest)
        next += (int64_t)(rng() % 3) * gale::OffsetWindow::kMaxSpan + (int64_t)(rng() % 5000);
      } else if (r < 95 && next > 50) {  // seek back a little (re-fetch)
        next -= (int64_t)(rng() % 50);
      } else if (!model.empty()) {
        w.done(*model.begin());
        model.erase(model.begin());
      }
      if (w.empty() != model.empty()) {
        fprintf(stderr, "round %d step %d: empty %d vs %d\n", round, step, w.empty(),
                model.empty());
        return 1;
      }
      if (!model.empty() && w.first() != *model.begin()) {
        fprintf(stderr, "round %d step %d: first %lld vs %lld\n", round, step,
                (long long)w.first(), (long long)*model.begin());
        return 1;
      }
      if ((int64_t)w.st.size() > gale::OffsetWindow::kMaxSpan + 1) {
        fprintf(stderr, "window span %zu over the bound\n", w.st.size());
        return 1;
      }
    }
  }
  printf("offset window OK\n");
  return 0;
}
