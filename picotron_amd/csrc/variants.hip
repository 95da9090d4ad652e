// Measurement variants of the kernel library (include/picotron_hip.h, pt_set_variant): one table per
// process, written by the host, read by the launchers.  No environment is read anywhere in csrc/.
#include <string.h>

#include "common.h"

namespace {
struct VariantDef { const char* name; int value; };
VariantDef g_variants[PT_VAR_COUNT] = {
    {"attn_pair", 1}, {"attn_split", 2}, {"gemm_mix", 1}, {"gemm_kh", 2}, {"attn_kv_chunk", 4}};

int find(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < PT_VAR_COUNT; ++i)
    if (strcmp(g_variants[i].name, name) == 0) return i;
  return -1;
}
}  // namespace

int pt_variant(PtVariant v) { return g_variants[v].value; }

extern "C" {

int pt_set_variant(const char* name, int value) {
  const int i = find(name);
  if (i < 0) return PT_EINVAL;
  g_variants[i].value = value;
  return PT_OK;
}

int pt_get_variant(const char* name) {
  const int i = find(name);
  return i < 0 ? PT_EINVAL : g_variants[i].value;
}

}  // extern "C"
