// Host build of clonos_amd/csrc/handoff.h for tests/test_handoff_words.py (hipcc
// --offload-host-only): the polled-word encoding the fused decode uses, behind a C ABI.
#include "../clonos_amd/csrc/handoff.h"

extern "C" {
uint64_t ho_word(uint32_t state, uint64_t v) { return clg::pk_word(state, v); }
uint32_t ho_state(uint64_t w) { return clg::pk_state(w); }
uint64_t ho_val(uint64_t w) { return clg::pk_val(w); }
}
