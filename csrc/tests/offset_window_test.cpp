// OffsetWindow (csrc/runtime/engine.h) against a std::set model: random adds / completions with
// seeks back and far forward jumps; the oldest pending offset (the commit position) must always
// agree and the window must stay within its span bound. Built and run by
// tests/test_offset_window.py (host code only).
#include <stdio.h>

#include <random>
#include <set>

#include "../runtime/engine.h"

int main() {
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
