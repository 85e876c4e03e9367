// The one instance of rt::Tuning (csrc/include/rt_tuning.h): read by the launchers, written only
// through rt_set_tuning (the Python binding set_tuning).
#include "rt_tuning.h"

namespace {
rt::Tuning g_tuning;
}

extern "C" const rt::Tuning* rt_tuning() { return &g_tuning; }
extern "C" void rt_set_tuning(const rt::Tuning* t) {
  if (t) g_tuning = *t;
}
