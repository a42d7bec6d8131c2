// TEST/DEBUG TOOL ONLY: per-transition trace of the Check interpreter in the CPU emulation
// (tools/sim_regroup.py).  Byte stream: 0xFE + u32 start-record position at a query's first
// step, 0xFF at every later step boundary (load slot), one byte per transition (dispatch key).
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
inline FILE *keto_emu_trace_file() {
    static FILE *f = [] {
        const char *p = std::getenv("KETO_EMU_TRACE_FILE");
        return p ? std::fopen(p, "wb") : nullptr;
    }();
    return f;
}
inline void keto_emu_trace_step(uint32_t start_pos) {
    if (FILE *f = keto_emu_trace_file()) {
        if (start_pos != 0xFFFFFFFFu) {
            std::fputc(0xFE, f);
            std::fwrite(&start_pos, 4, 1, f);
        } else {
            std::fputc(0xFF, f);
        }
    }
}
inline void keto_emu_trace_key(uint32_t key) {
    if (FILE *f = keto_emu_trace_file()) std::fputc((int)key, f);
}
