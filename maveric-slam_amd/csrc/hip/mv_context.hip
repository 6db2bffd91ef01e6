// mv_context.hip -- context, stream, scratch and status plumbing of the C ABI.
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>

#include "mv_internal.hpp"

namespace {
thread_local int g_last_status = MV_OK;
thread_local char g_last_msg[512] = "";
// The default context is PER THREAD (the drop-in entry points keep the reference's
// single-threaded signatures, so the context is implicit): each host thread gets its own
// stream, staging and scratch, created on first use and destroyed when the thread exits
// (the main thread's lives until process exit).
pthread_once_t g_key_once = PTHREAD_ONCE_INIT;
pthread_key_t g_ctx_key;
std::atomic<bool> g_no_device_reported{false};

void destroy_thread_context(void *p) { (void)mv_context_destroy(static_cast<mv_context *>(p)); }
void make_key() { (void)pthread_key_create(&g_ctx_key, destroy_thread_context); }
}  // namespace

namespace mv {
void set_error(int status, const char *fmt, ...) {
    g_last_status = status;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_msg, sizeof g_last_msg, fmt, ap);
    va_end(ap);
}

int set_status(int status) {
    g_last_status = status;
    if (status == MV_OK) g_last_msg[0] = 0;
    return status;
}

int quiesce(mv_context *ctx) {
    // own_stream waits on every stream the context left (ev_retire), so these three cover all
    // of the context's work; every stream is synchronised even after a failure, and a failure
    // falls back to the whole device before the caller frees a buffer
    hipError_t e = hipStreamSynchronize(ctx->own_stream);
    if (ctx->stream != ctx->own_stream) {
        const hipError_t e2 = hipStreamSynchronize(ctx->stream);
        if (e == hipSuccess) e = e2;
    }
    if (ctx->aux_stream) {
        const hipError_t e3 = hipStreamSynchronize(ctx->aux_stream);
        if (e == hipSuccess) e = e3;
    }
    if (e != hipSuccess) {
        (void)hipDeviceSynchronize();
        set_error(MV_ERR_HIP, "quiesce: %s", hipGetErrorString(e));
        return MV_ERR_HIP;
    }
    return MV_OK;
}

// *cap = whether `s` is being captured into a graph.  A query refused with a capture error is also
// "capturing": that is what the legacy NULL stream answers while another stream captures in global
// mode, and no event may then be recorded on it or waited for by it (a record on the legacy stream,
// or an uncaptured event waited for by a capturing stream, invalidates the capture; a wait of
// own_stream on an event recorded inside a capture pulls own_stream into it, unjoined).  Any other
// refusal (an invalid or destroyed stream handle) is reported, not taken for a capture: skipping the
// event record / wait would leave the context's reused scratch unordered.
int capture_state(hipStream_t s, bool *cap) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    const hipError_t e = hipStreamIsCapturing(s, &st);
    if (e == hipSuccess) {
        *cap = st != hipStreamCaptureStatusNone;
        return MV_OK;
    }
    (void)hipGetLastError();  // clear the sticky query error
    if (e == hipErrorStreamCaptureImplicit || e == hipErrorStreamCaptureUnsupported ||
        e == hipErrorStreamCaptureInvalidated || e == hipErrorStreamCaptureWrongThread) {
        *cap = true;
        return MV_OK;
    }
    *cap = false;
    set_error(MV_ERR_HIP, "hipStreamIsCapturing: %s", hipGetErrorString(e));
    return MV_ERR_HIP;
}

// the context moves off `old`: own_stream waits for everything issued on it so far (not when
// `old` is being captured: the graph's launches are the caller's to order, see maveric_hip.h)
static int retire_stream(mv_context *ctx, hipStream_t old) {
    if (old == ctx->own_stream) return MV_OK;
    bool cap = false;
    const int rc = capture_state(old, &cap);
    if (rc != MV_OK || cap) return rc;
    if (!ctx->ev_retire) MV_HIP_TRY(hipEventCreateWithFlags(&ctx->ev_retire, hipEventDisableTiming));
    MV_HIP_TRY(hipEventRecord(ctx->ev_retire, old));
    MV_HIP_TRY(hipStreamWaitEvent(ctx->own_stream, ctx->ev_retire, 0));
    return MV_OK;
}

void *scratch(mv_context *ctx, size_t bytes) {
    if (bytes <= ctx->scratch_bytes) return ctx->scratch;
    if (ctx->scratch) {
        (void)quiesce(ctx);  // the old buffer may be in use on any stream the context used
        (void)hipFree(ctx->scratch);
        ctx->scratch = nullptr;
        ctx->scratch_bytes = 0;
    }
    size_t b = align_up(bytes, 1 << 20);
    if (hipMalloc(&ctx->scratch, b) != hipSuccess) {
        set_error(MV_ERR_OUT_OF_MEMORY, "scratch allocation of %zu bytes failed", b);
        ctx->scratch = nullptr;
        return nullptr;
    }
    ctx->scratch_bytes = b;
    return ctx->scratch;
}

void *stage(mv_context *ctx, size_t bytes) {
    if (bytes <= ctx->stage_bytes) return ctx->stage_dev;
    if (ctx->stage_dev) {
        (void)quiesce(ctx);
        (void)hipFree(ctx->stage_dev);
        ctx->stage_dev = nullptr;
        ctx->stage_bytes = 0;
    }
    size_t b = align_up(bytes, 1 << 20);
    if (hipMalloc(&ctx->stage_dev, b) != hipSuccess) {
        set_error(MV_ERR_OUT_OF_MEMORY, "staging allocation of %zu bytes failed", b);
        ctx->stage_dev = nullptr;
        return nullptr;
    }
    ctx->stage_bytes = b;
    return ctx->stage_dev;
}
}  // namespace mv

extern "C" {

int mv_version(void) { return MV_VERSION; }

const char *mv_status_string(int s) {
    switch (s) {
        case MV_OK: return "ok";
        case MV_ERR_INVALID_ARG: return "invalid argument";
        case MV_ERR_CAPACITY: return "capacity exceeded";
        case MV_ERR_HIP: return "HIP runtime error";
        case MV_ERR_NO_DEVICE: return "no HIP device";
        case MV_ERR_NO_POINTS: return "no correspondences";
        case MV_ERR_OUT_OF_MEMORY: return "out of device memory";
        case MV_ERR_DEGENERATE: return "degenerate pose";
        case MV_ERR_IO: return "file I/O error";
        default: return "unknown status";
    }
}

int mv_last_status(void) { return g_last_status; }
const char *mv_last_error_message(void) { return g_last_msg; }

int mv_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int mv_context_create(int device, mv_context **out) {
    MV_REQUIRE(out != nullptr);
    *out = nullptr;
    int n = mv_device_count();
    if (device < 0 || device >= n) {
        mv::set_error(MV_ERR_NO_DEVICE, "device %d requested, %d visible", device, n);
        return MV_ERR_NO_DEVICE;
    }
    hipDeviceProp_t prop;
    MV_HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        mv::set_error(MV_ERR_NO_DEVICE, "device %d is %s, this build targets gfx950 only", device,
                      prop.gcnArchName);
        return MV_ERR_NO_DEVICE;
    }
    MV_HIP_TRY(hipSetDevice(device));
    mv_context *c = new mv_context();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        mv::set_error(MV_ERR_HIP, "hipStreamCreate failed");
        return MV_ERR_HIP;
    }
    c->stream = c->own_stream;
    const char *scr = getenv("MV_AP_SCREEN");
    c->ap_screen = (scr && strcmp(scr, "f16") == 0)   ? MV_SCREEN_F16
                   : (scr && strcmp(scr, "i8s") == 0) ? MV_SCREEN_I8_STAGED
                                                      : MV_SCREEN_I8;
    *out = c;
    return mv::set_status(MV_OK);
}

int mv_context_destroy(mv_context *ctx) {
    if (!ctx) return MV_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->aux_stream) {
        (void)hipStreamSynchronize(ctx->aux_stream);
        (void)hipEventDestroy(ctx->ev_in);
        (void)hipEventDestroy(ctx->ev_prep);
        (void)hipStreamDestroy(ctx->aux_stream);
    }
    (void)hipStreamSynchronize(ctx->own_stream);  // the streams the context left (ev_retire)
    if (ctx->ev_retire) (void)hipEventDestroy(ctx->ev_retire);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->ap_scratch) (void)hipFree(ctx->ap_scratch);
    if (ctx->ap_scratch2) (void)hipFree(ctx->ap_scratch2);
    if (ctx->stage_dev) (void)hipFree(ctx->stage_dev);
    if (ctx->i8_count_host) (void)hipHostFree(ctx->i8_count_host);
    (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return MV_OK;
}

int mv_context_set_stream(mv_context *ctx, void *s) {
    MV_REQUIRE(ctx != nullptr);
    bool cap_new = false;
    if ((hipStream_t)s != ctx->stream) {
        const int rc = mv::capture_state((hipStream_t)s, &cap_new);
        if (rc != MV_OK) return rc;
    }
    if ((hipStream_t)s != ctx->stream && cap_new) {
        // onto a capture stream: no event on either stream (a record on the legacy NULL stream
        // during a global-mode capture invalidates it); the caller has synchronised before capturing
        ctx->stream = (hipStream_t)s;
        return MV_OK;
    }
    if ((hipStream_t)s != ctx->stream) {
        MV_HIP_TRY(hipSetDevice(ctx->device));
        const int r = mv::retire_stream(ctx, ctx->stream);
        if (r != MV_OK) return r;
        // the new stream also orders after the old one: the context's buffers (scratch, staged
        // images) are reused by its next launch.  Not across a capture: entering one, the caller
        // has ordered the capture stream after the earlier work (a capture cannot wait for an
        // uncaptured event); leaving one, nothing outside the graph can wait for it.
        bool cap_old = false;
        const int rc = mv::capture_state(ctx->stream, &cap_old);
        if (rc != MV_OK) return rc;
        if (!cap_old) {
            if (!ctx->ev_retire) MV_HIP_TRY(hipEventCreateWithFlags(&ctx->ev_retire, hipEventDisableTiming));
            MV_HIP_TRY(hipEventRecord(ctx->ev_retire, ctx->stream));
            MV_HIP_TRY(hipStreamWaitEvent((hipStream_t)s, ctx->ev_retire, 0));
        }
    }
    ctx->stream = (hipStream_t)s;  // NULL is HIP's null stream (torch's default stream), not "unset"
    return MV_OK;
}

int mv_context_use_own_stream(mv_context *ctx) {
    MV_REQUIRE(ctx != nullptr);
    if (ctx->stream != ctx->own_stream) {
        MV_HIP_TRY(hipSetDevice(ctx->device));
        const int r = mv::retire_stream(ctx, ctx->stream);
        if (r != MV_OK) return r;
    }
    ctx->stream = ctx->own_stream;
    return MV_OK;
}

void *mv_context_stream(mv_context *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int mv_context_synchronize(mv_context *ctx) {
    MV_REQUIRE(ctx != nullptr);
    MV_HIP_TRY(hipStreamSynchronize(ctx->stream));
    return MV_OK;
}

int mv_context_set_allpairs_screen(mv_context *ctx, int screen) {
    MV_REQUIRE(ctx != nullptr && (screen == MV_SCREEN_I8 || screen == MV_SCREEN_F16 || screen == MV_SCREEN_I8_STAGED));
    ctx->ap_screen = screen;
    return MV_OK;
}

int mv_context_allpairs_screen(mv_context *ctx) { return ctx ? ctx->ap_screen : MV_ERR_INVALID_ARG; }

int mv_context_reserve(mv_context *ctx, int batch, int cap) {
    MV_REQUIRE(ctx != nullptr && batch > 0 && cap > 0);
    // the staged images of the context's CURRENT screen (ap_image_bytes) and run_prepare's second
    // image; the default one-pass int8 screen stages nothing (sequence mode allocates its images
    // on first use)
    const size_t img = ctx->ap_screen == MV_SCREEN_I8 ? 0 : mv::ap_image_bytes(ctx->ap_screen, batch, cap);
    if (img && ctx->ap_scratch_bytes < img) {
        if (ctx->ap_scratch) {
            const int q = mv::quiesce(ctx);
            if (q != MV_OK) return q;
            MV_HIP_TRY(hipFree(ctx->ap_scratch));
            ctx->ap_scratch = nullptr;
            ctx->ap_scratch_bytes = 0;
        }
        ctx->prep_desc1 = nullptr;  // a prepared frame 1 lived in the freed buffer
        const size_t ab = mv::align_up(img, 1 << 20);
        if (hipMalloc(&ctx->ap_scratch, ab) != hipSuccess) return MV_ERR_OUT_OF_MEMORY;
        ctx->ap_scratch_bytes = ab;
    }
    if (img && ctx->ap_scratch2_bytes < img) {  // run_prepare's second image
        if (ctx->ap_scratch2) {
            const int q = mv::quiesce(ctx);
            if (q != MV_OK) return q;
            MV_HIP_TRY(hipFree(ctx->ap_scratch2));
            ctx->ap_scratch2 = nullptr;
            ctx->ap_scratch2_bytes = 0;
        }
        const size_t ab = mv::align_up(img, 1 << 20);
        if (hipMalloc(&ctx->ap_scratch2, ab) != hipSuccess) return MV_ERR_OUT_OF_MEMORY;
        ctx->ap_scratch2_bytes = ab;
    }
    size_t need = mv::allpairs_i8_scratch_bytes(batch, cap);
    size_t b;
    b = mv::pose_scratch_bytes(batch, cap);
    if (b > need) need = b;
    if (!mv::scratch(ctx, need)) return MV_ERR_OUT_OF_MEMORY;
    return MV_OK;
}

mv_context *mv_default_context(void) {
    pthread_once(&g_key_once, make_key);
    mv_context *c = static_cast<mv_context *>(pthread_getspecific(g_ctx_key));
    if (c) {
        (void)hipSetDevice(c->device);
        return c;
    }
    const int n = mv_device_count();
    if (n <= 0) {
        if (!g_no_device_reported.exchange(true))
            fprintf(stderr,
                    "maveric_hip: no HIP device visible -- this library has no CPU fallback "
                    "(hipGetDeviceCount = %d)\n", n);
        mv::set_error(MV_ERR_NO_DEVICE, "no HIP device visible");
        return nullptr;
    }
    if (mv_context_create(0, &c) != MV_OK) {
        fprintf(stderr, "maveric_hip: cannot create the default context: %s\n", g_last_msg);
        return nullptr;
    }
    (void)pthread_setspecific(g_ctx_key, c);
    return c;
}

}  // extern "C"
