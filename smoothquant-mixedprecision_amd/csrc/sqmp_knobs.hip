// Launch-variant knobs (the SQMP_* A/B and tuning variables of DESIGN.md §7): read ONCE, when
// the library is loaded, into a table; the launchers look values up there instead of calling
// getenv per launch.  sqmp_reload_knobs() re-reads the environment: the in-process A/B tools
// (tools/ab_*.py, tools/step_ab.py) and the tests that switch a variant call it after changing
// os.environ.  Every launcher reads its knob through knob() at each launch (no launcher caches
// a value), so a reload reaches all of them.  Values live in fixed per-knob buffers that are
// never freed: a pointer knob() returned stays valid (a reload concurrent with a launch on
// another thread may at worst hand that launch the old or the new value).
#include <stdlib.h>
#include <string.h>

#include "sqmp_internal.h"

namespace sqmp {

static const char* const kKnobs[] = {
    "SQMP_NT_STORES",   "SQMP_RANK_TABLE_OFF", "SQMP_RT_TPO",      "SQMP_RT_R",
    "SQMP_RT_SB",       "SQMP_RT_BUCKET",      "SQMP_RT_DENSE",      "SQMP_RT_K16", "SQMP_RT_HIST",      "SQMP_RT_BTPO",     "SQMP_DISABLE_LC",
    "SQMP_LC_PERCU",    "SQMP_PW_RB",          "SQMP_C4_QPERCU",   "SQMP_F32_WN2",
    "SQMP_F8_V1",       "SQMP_GROUP_M",        "SQMP_F8_OPT",      "SQMP_F8_DIAG",     "SQMP_F8_TM",
    "SQMP_FQ7_GROUP_M", "SQMP_FQT7_GROUP_M",   "SQMP_FQ7_OPT",     "SQMP_FQT7_OPT",
    "SQMP_FQ7_DIAG",    "SQMP_FQ7G_TM", "SQMP_FQ7_KS",        "SQMP_H2D_GROUP_M", "SQMP_H2_WIDE",
    "SQMP_H2_BK64",     "SQMP_H2_GROUP_M",     "SQMP_COLMAX_RPB",  "SQMP_LC_PPW",
};
constexpr int NKNOBS = (int)(sizeof(kKnobs) / sizeof(kKnobs[0]));
constexpr int KNOB_LEN = 32;  // every knob is a short integer or name
static char g_val[NKNOBS][KNOB_LEN];
static const char* volatile g_knob[NKNOBS];

static void load_knobs() {
  for (int i = 0; i < NKNOBS; ++i) {
    const char* e = getenv(kKnobs[i]);
    if (!e) {
      g_knob[i] = nullptr;
      continue;
    }
    strncpy(g_val[i], e, KNOB_LEN - 1);  // (the last byte stays 0)
    g_knob[i] = g_val[i];
  }
}

__attribute__((constructor)) static void knobs_at_load() { load_knobs(); }

const char* knob(const char* name) {
  for (int i = 0; i < NKNOBS; ++i)
    if (strcmp(name, kKnobs[i]) == 0) return (const char*)g_knob[i];
  return nullptr;  // (a name missing from the table reads as unset)
}

}  // namespace sqmp

extern "C" int sqmp_reload_knobs(void) {
  sqmp::load_knobs();
  return SQMP_OK;
}
