// TEST/DEBUG TOOL ONLY (compiled into the CPU emulation library, never into the product): a probe
// of the scratch cache's stream discipline.  A builder temporary released while a keto_stream's
// streams are the thread's scratch stream carries an event recorded on that stream; the stream
// object is then destroyed, and the same-sized block is taken again.  With the emulation's stream
// liveness (hip/hip_runtime.h) that take fails unless keto_stream_destroy retired the event first.
#include "../../djy-keto_amd/csrc/engine.hpp"

extern "C" int keto_emu_scratch_dead_stream_probe(void) {
    try {
        keto_stream *ks = nullptr;
        if (keto_stream_create(0, &ks) != KETO_OK) return -100;
        keto::Stream *st = reinterpret_cast<keto::Stream *>(ks);
        KETO_HIP(hipStreamCreateWithFlags(&st->h2d, hipStreamNonBlocking));  // (as an async batch creates them)
        KETO_HIP(hipStreamCreateWithFlags(&st->d2h, hipStreamNonBlocking));
        const size_t sizes[3] = {(size_t)3 << 20, (size_t)5 << 20, (size_t)7 << 20};
        hipStream_t on[3] = {st->stream, st->h2d, st->d2h};
        for (int i = 0; i < 3; i++) {
            keto::ScratchStream scope(on[i]);
            keto::build::DevBuf b(sizes[i]);  // released at the end of the scope: its event is on on[i]
        }
        keto_stream_destroy(ks);
        for (int i = 0; i < 3; i++) {
            size_t got = 0;
            void *p = keto::scratch_get(sizes[i] + 16, &got);  // (DevBuf asks for bytes + 16)
            keto::scratch_put(p, got);
        }
        return 0;
    } catch (const keto::Error &e) {
        return e.code;
    }
}
