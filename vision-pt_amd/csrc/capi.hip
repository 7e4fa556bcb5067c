// C-ABI bookkeeping for libvpt_hip.so: thread-local last-error string and library info.
// See include/vpt_hip.h for the full entry-point list.
#include <cstdio>
#include <cstring>
#include "common.h"

namespace {
thread_local char g_err[512] = "";
}

extern "C" void vpt_set_error(const char* msg) {
  std::strncpy(g_err, msg ? msg : "", sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = '\0';
}

extern "C" const char* vpt_last_error_string(void) { return g_err; }

// 2: attention takes nk (cross-attention). 3: vpt_radam_sf_step takes (clip_coef, clip_value) before the stream and
// vpt_ema_update takes one_minus_decay before `first` -- a caller built against ABI 2 must not bind ABI 3.
// ABI 4: vpt_embed_grad_set takes `accumulate` before dtable.
// ABI 5: vpt_geglu_bwd_lora takes tickets + partials (vpt_geglu_lora_partials_bytes).
#define VPT_ABI_VERSION 5
#define VPT_STR2(x) #x
#define VPT_STR(x) VPT_STR2(x)
extern "C" int vpt_abi_version(void) { return VPT_ABI_VERSION; }

extern "C" const char* vpt_build_info(void) { return "vpt_hip gfx950 (CDNA4) bf16-MFMA abi=" VPT_STR(VPT_ABI_VERSION); }
