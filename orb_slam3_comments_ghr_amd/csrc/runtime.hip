#include <string>
// runtime.hip — context lifecycle, scratch pool, errors (C ABI: include/osg.h "context").
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <cstring>

#include "osg_internal.h"

#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <unistd.h>

#include <condition_variable>
#include <deque>
#include <mutex>

namespace {
// the cgroup (v2 cpu.max, else v1 cfs) CPU quota in whole CPUs, rounded up; 0 when unlimited
int cgroup_cpus()
{
    long long quota = -1, period = 0;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {};
        if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0) quota = atoll(q);
        fclose(f);
    } else if (FILE *f1 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
        if (fscanf(f1, "%lld", &quota) != 1) quota = -1;
        fclose(f1);
        if (FILE *f2 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
            if (fscanf(f2, "%lld", &period) != 1) period = 0;
            fclose(f2);
        }
    }
    return quota > 0 && period > 0 ? (int)((quota + period - 1) / period) : 0;
}
// CPUs of the cgroup's cpuset (v2 cpuset.cpus.effective, else v1 cpuset.effective_cpus, a cpulist such
// as "0-15,32-47"); 0 when neither is readable
int cpuset_cpus()
{
    const char *paths[] = {"/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/cpuset/cpuset.effective_cpus"};
    for (const char *p : paths) {
        FILE *f = fopen(p, "r");
        if (!f) continue;
        char buf[4096] = {};
        const size_t len = fread(buf, 1, sizeof(buf) - 1, f);
        fclose(f);
        buf[len] = 0;
        int n = 0;
        for (char *s = buf; *s && *s != '\n';) {
            char *e = nullptr;
            const long a = strtol(s, &e, 10);
            if (e == s) break;
            long b = a;
            if (*e == '-') {
                s = e + 1;
                b = strtol(s, &e, 10);
            }
            if (b >= a) n += (int)(b - a + 1);
            s = (*e == ',') ? e + 1 : e;
        }
        if (n > 0) return n;
    }
    return 0;
}
// the worker pool behind osg_parallel_run
struct PoolJob {
    void (*fn)(void *, int);
    void *arg;
    int n;
    std::atomic<int> next{0}, done{0}, active{0};
    int seats;  // workers that may still join (under the pool's mutex)
    // the owner sleeps on this after a short spin; the thread that finishes the last index wakes it
    std::mutex m;
    std::condition_variable cv;
};
struct WorkerPool {
    std::mutex m;
    std::condition_variable cv;
    std::deque<PoolJob *> q;
    std::vector<std::thread> th;
    explicit WorkerPool(int nw)
    {
        for (int i = 0; i < nw; i++) th.emplace_back([this] { loop(); });
        for (auto &t : th) t.detach();  // live for the process (never torn down at exit)
    }
    static void run(PoolJob *j)
    {
        for (int i = j->next++; i < j->n; i = j->next++) {
            j->fn(j->arg, i);
            if (++j->done == j->n) {
                std::lock_guard<std::mutex> lk(j->m);
                j->cv.notify_all();
            }
        }
    }
    void loop()
    {
        for (;;) {
            PoolJob *j = nullptr;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] {
                    for (PoolJob *c : q)
                        if (c->seats > 0 && c->next.load() < c->n) return true;
                    return false;
                });
                for (PoolJob *c : q)
                    if (c->seats > 0 && c->next.load() < c->n) {
                        c->seats--;
                        c->active++;  // under the mutex: the owner removes the job under it too
                        j = c;
                        break;
                    }
            }
            if (!j) continue;
            run(j);
            j->active--;  // the worker's last access to the job
        }
    }
};
WorkerPool *pool()
{
    // no loop asks for more than 16 threads
    static WorkerPool *p = new WorkerPool(std::max(0, std::min(osg_host_cpus(), 16) - 1));
    return p;
}
}  // namespace

int osg_host_cpus()
{
    static const int n = [] {
        if (const char *e = getenv("OSG_HOST_THREADS"))
            if (atoi(e) > 0) return atoi(e);
        const int hw = std::max(1, (int)std::thread::hardware_concurrency());
        int c = hw, aff = hw;
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) {
            aff = std::max(1, CPU_COUNT(&set));
            c = std::min(c, aff);
        }
        const int q = cgroup_cpus();
        if (q > 0) c = std::min(c, q);
        // one process per GPU (torchrun): the node's share is split between the local ranks, unless
        // the launcher already pinned each rank to its own share (not divided twice).  A rank
        // counts as pinned only when its affinity set is at most its 1 / LOCAL_WORLD_SIZE part of the
        // set all local ranks share (the cgroup's cpuset, else the machine): a container's cpuset that
        // every rank inherits is smaller than the machine but is not a per-rank pinning
        if (const char *lwe = getenv("LOCAL_WORLD_SIZE")) {
            const int lw = atoi(lwe);
            if (lw > 1) {
                const int cs = cpuset_cpus();
                const int shared = cs > 0 ? std::min(cs, hw) : hw;
                const bool pinned = (long long)aff * lw <= shared;
                if (!pinned) c = std::max(1, c / lw);
            }
        }
        return c;
    }();
    return n;
}

void osg_parallel_run(int n, int max_threads, void (*fn)(void *, int), void *arg)
{
    if (n <= 0) return;
    PoolJob j;
    j.fn = fn;
    j.arg = arg;
    j.n = n;
    WorkerPool *p = n > 1 && max_threads > 1 ? pool() : nullptr;
    j.seats = p ? std::min(std::min(n, max_threads) - 1, (int)p->th.size()) : 0;
    const bool queued = j.seats > 0;
    if (queued) {
        {
            std::lock_guard<std::mutex> lk(p->m);
            p->q.push_back(&j);
        }
        p->cv.notify_all();
    }
    WorkerPool::run(&j);
    if (queued) {  // the job lives on this stack: out of the queue and no worker inside before returning
        // spin briefly (most loops end within it), then sleep until the last index is done, so a
        // caller waiting on a long index does not burn a core beside the pool's workers
        const auto t0 = std::chrono::steady_clock::now();
        while (j.done.load() < n &&
               std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < 50.0)
            std::this_thread::yield();
        if (j.done.load() < n) {
            std::unique_lock<std::mutex> lk(j.m);
            j.cv.wait(lk, [&] { return j.done.load() >= n; });
        }
        {
            std::lock_guard<std::mutex> lk(p->m);
            for (auto it = p->q.begin(); it != p->q.end(); ++it)
                if (*it == &j) {
                    p->q.erase(it);
                    break;
                }
        }
        while (j.active.load() > 0) std::this_thread::yield();
    }
}

int osg_set_error(osg_ctx *ctx, int code, const char *fmt, ...)
{
    if (ctx) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        ctx->last_error = buf;
    }
    return code;
}

void *osg_scratch(osg_ctx *ctx, int slot, size_t bytes)
{
    if (bytes == 0) bytes = 16;
    if (ctx->cap[slot] >= bytes) return ctx->buf[slot];
    if (ctx->buf[slot]) {
        // the previous buffer may still be read by queued work on this stream
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(ctx->buf[slot]);
        ctx->buf[slot] = nullptr;
        ctx->cap[slot] = 0;
    }
    size_t cap = bytes + bytes / 4 + 256;
    cap = (cap + 255) & ~size_t(255);
    void *p = nullptr;
    if (hipMalloc(&p, cap) != hipSuccess) return nullptr;
    ctx->buf[slot] = p;
    ctx->cap[slot] = cap;
    return p;
}

hipEvent_t *osg_ctx_events(osg_ctx *ctx)
{
    if (!ctx->ev[0]) {
        if (hipEventCreate(&ctx->ev[0]) != hipSuccess || hipEventCreate(&ctx->ev[1]) != hipSuccess) return nullptr;
    }
    return ctx->ev;
}

void *osg_pinned(osg_ctx *ctx, size_t bytes)
{
    if (ctx->host_pinned_cap >= bytes) return ctx->host_pinned;
    if (ctx->host_pinned) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipHostFree(ctx->host_pinned);
        ctx->host_pinned = nullptr;
        ctx->host_pinned_cap = 0;
    }
    size_t cap = bytes + bytes / 4 + 4096;
    void *p = nullptr;
    // coherent (fine-grained) pages: k_copy loads and stores them directly, and each call's upload /
    // download must see the host's latest bytes at the same offsets with no stale GPU L2 line, whatever
    // fence scope the runtime gives the dispatch (HIP_HOST_COHERENT is not relied on)
    if (hipHostMalloc(&p, cap, hipHostMallocCoherent) != hipSuccess) return nullptr;
    ctx->host_pinned = p;
    ctx->host_pinned_cap = cap;
    return p;
}

// Why a kernel for small transfers: an SDMA copy on the stream makes the next kernel wait for the
// copy engine's completion signal; rocprofv3 --hip-trace of a one-frame SearchByBoW showed the first
// kernel starting 12 us after its upload had finished, and the download, a blit kernel the runtime
// inserts for pinned destinations, starting 6 us after the last kernel.  A copy kernel is ordered like
// any other launch in the queue.  16 bytes per thread per step; the pinned and scratch buffers are
// 256-byte aligned and callers pass aligned offsets, so only the byte tail is moved singly.
namespace {
__global__ __launch_bounds__(256) void k_copy(uint4 *__restrict__ dst, const uint4 *__restrict__ src, size_t n16,
                                              unsigned char *__restrict__ dtail,
                                              const unsigned char *__restrict__ stail, int ntail)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < ntail) dtail[threadIdx.x] = stail[threadIdx.x];
}

bool in_pinned(const osg_ctx *ctx, const void *p, size_t bytes)
{
    const char *b = (const char *)ctx->host_pinned, *q = (const char *)p;
    return b && q >= b && q + bytes <= b + ctx->host_pinned_cap;
}

int kcopy(osg_ctx *ctx, void *dst, const void *src, size_t bytes)
{
    const size_t n16 = ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) ? bytes / 16 : 0;
    const int ntail = (int)(bytes - 16 * n16);
    if (ntail > 256) return -1;  // misaligned: the caller falls back to the copy engine
    const int blocks = (int)std::min<size_t>(std::max<size_t>((n16 + 255) / 256, 1), 1024);
    hipLaunchKernelGGL(k_copy, dim3(blocks), dim3(256), 0, ctx->stream, (uint4 *)dst, (const uint4 *)src, n16,
                       (unsigned char *)dst + 16 * n16, (const unsigned char *)src + 16 * n16, ntail);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    return OSG_OK;
}
}  // namespace

int osg_upload(osg_ctx *ctx, void *dst_dev, const void *src_pinned, size_t bytes)
{
    if (bytes == 0) return OSG_OK;
    if (bytes <= OSG_KCOPY_MAX && in_pinned(ctx, src_pinned, bytes)) {
        const int rc = kcopy(ctx, dst_dev, src_pinned, bytes);
        if (rc != -1) return rc;
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dst_dev, src_pinned, bytes, hipMemcpyHostToDevice, ctx->stream));
    return OSG_OK;
}

int osg_download(osg_ctx *ctx, void *dst_pinned, const void *src_dev, size_t bytes)
{
    if (bytes == 0) return OSG_OK;
    if (bytes <= OSG_KCOPY_MAX && in_pinned(ctx, dst_pinned, bytes)) {
        const int rc = kcopy(ctx, dst_pinned, src_dev, bytes);
        if (rc != -1) return rc;
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dst_pinned, src_dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
    return OSG_OK;
}

int osg_idle(osg_ctx *ctx)
{
    if (hipStreamQuery(ctx->stream) == hipSuccess) return OSG_OK;
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return OSG_OK;
}

// Wait for the stream: poll its completion event for up to OSG_WAIT_SPIN_US microseconds (default
// 100: a one-frame matcher call ends within that, and returns ~1 us after its last kernel), then
// block on the event (created with hipEventBlockingSync, so the thread sleeps instead of burning a
// host core that Tracking / LocalMapping / LoopClosing threads need while a long BA call runs).
int osg_wait(osg_ctx *ctx)
{
    // OSG_WAIT=sync: a stream synchronisation instead of the polled event (A/B runs)
    static const bool sync_wait = getenv("OSG_WAIT") && std::string(getenv("OSG_WAIT")) == "sync";
    static const double spin_us = getenv("OSG_WAIT_SPIN_US") ? atof(getenv("OSG_WAIT_SPIN_US")) : 100.0;
    if (sync_wait) {
        OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
        return OSG_OK;
    }
    if (!ctx->ev_done &&
        hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) {
        ctx->ev_done = nullptr;
        OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
        return OSG_OK;
    }
    OSG_HIP_CHECK(ctx, hipEventRecord(ctx->ev_done, ctx->stream));
    const auto t0 = std::chrono::steady_clock::now();
    for (int it = 0;; it++) {
        const hipError_t e = hipEventQuery(ctx->ev_done);
        if (e == hipSuccess) return OSG_OK;
        if (e != hipErrorNotReady)
            return osg_set_error(ctx, OSG_E_HIP, "hipEventQuery failed: %s", hipGetErrorString(e));
        if ((it & 15) == 15 &&
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > spin_us)
            break;
        __builtin_ia32_pause();
    }
    OSG_HIP_CHECK(ctx, hipEventSynchronize(ctx->ev_done));
    return OSG_OK;
}

// OSG_SEGV_MAPS=1: on SIGSEGV / SIGBUS, write the faulting address and /proc/self/maps to stderr, then
// hand the signal to the handler installed before ours (e.g. a profiler's stack dumper), so a native
// stack trace of unsymbolised frames can be mapped to libraries afterwards.  Only
// open / read / write are used inside the handler (async-signal-safe).
namespace {
struct sigaction g_prev_segv, g_prev_bus;

void write_all(int fd, const char *p, size_t n)
{
    while (n > 0) {
        const ssize_t w = write(fd, p, n);
        if (w <= 0) return;
        p += w;
        n -= (size_t)w;
    }
}

void maps_handler(int sig, siginfo_t *si, void *uc)
{
    char hdr[96];
    const int n = snprintf(hdr, sizeof hdr, "\n[osg] signal %d at %p; /proc/self/maps follows\n", sig,
                           si ? si->si_addr : nullptr);
    write_all(2, hdr, n > 0 ? (size_t)n : 0);
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        char buf[4096];
        for (ssize_t r; (r = read(fd, buf, sizeof buf)) > 0;) write_all(2, buf, (size_t)r);
        close(fd);
    }
    write_all(2, "[osg] end of maps\n", 18);
    struct sigaction &prev = sig == SIGBUS ? g_prev_bus : g_prev_segv;
    sigaction(sig, &prev, nullptr);  // the previous handler (or the default) takes the re-raised signal
    if ((prev.sa_flags & SA_SIGINFO) && prev.sa_sigaction) prev.sa_sigaction(sig, si, uc);
    else if (prev.sa_handler != SIG_IGN && prev.sa_handler != SIG_DFL) prev.sa_handler(sig);
    else raise(sig);
}

__attribute__((constructor)) void install_maps_handler()
{
    const char *e = getenv("OSG_SEGV_MAPS");
    if (!e || atoi(e) != 1) return;
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = maps_handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGBUS, &sa, &g_prev_bus);
}
}  // namespace

extern "C" {

const char *osg_version(void) { return "osg 0.1 gfx950 (orb_slam3_comments_ghr_amd)"; }

const char *osg_strerror(int code)
{
    switch (code) {
    case OSG_OK: return "ok";
    case OSG_E_INVALID: return "invalid argument";
    case OSG_E_HIP: return "HIP runtime error";
    case OSG_E_NOMEM: return "device allocation failed";
    case OSG_E_UNSUPPORTED: return "unsupported configuration";
    case OSG_E_NODEVICE: return "no gfx950 device";
    default: return code >= 0 ? "ok" : "unknown error";
    }
}

int osg_ctx_create(int device, osg_ctx **out)
{
    if (!out) return OSG_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return OSG_E_NODEVICE;
    if (device < 0 || device >= n) return OSG_E_INVALID;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return OSG_E_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return OSG_E_NODEVICE;
    if (hipSetDevice(device) != hipSuccess) return OSG_E_HIP;
    osg_ctx *ctx = new osg_ctx();
    ctx->device = device;
    ctx->num_cus = prop.multiProcessorCount;
    ctx->lds_per_block = (int)prop.sharedMemPerBlock;
    if (hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return OSG_E_HIP;
    }
    ctx->stream = ctx->own_stream;
    if (hipMalloc(&ctx->counters, sizeof(uint32_t) * OSG_N_COUNTERS) != hipSuccess ||
        hipMemset(ctx->counters, 0, sizeof(uint32_t) * OSG_N_COUNTERS) != hipSuccess) {
        (void)hipStreamDestroy(ctx->own_stream);
        delete ctx;
        return OSG_E_NOMEM;
    }
    *out = ctx;
    return OSG_OK;
}

int osg_ctx_destroy(osg_ctx *ctx)
{
    if (!ctx) return OSG_E_INVALID;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (int i = 0; i < SLOT_COUNT; i++)
        if (ctx->buf[i]) (void)hipFree(ctx->buf[i]);
    if (ctx->host_pinned) (void)hipHostFree(ctx->host_pinned);
    if (ctx->counters) (void)hipFree(ctx->counters);
    for (hipEvent_t e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->ev_done) (void)hipEventDestroy(ctx->ev_done);
    if (ctx->lb_flags) (void)hipFree(ctx->lb_flags);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return OSG_OK;
}

int osg_ctx_set_stream(osg_ctx *ctx, void *hip_stream)
{
    if (!ctx) return OSG_E_INVALID;
    ctx->stream = hip_stream ? (hipStream_t)hip_stream : ctx->own_stream;
    return OSG_OK;
}

void *osg_ctx_stream(osg_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int osg_ctx_synchronize(osg_ctx *ctx)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return OSG_OK;
}

const char *osg_ctx_last_error(osg_ctx *ctx) { return ctx ? ctx->last_error.c_str() : ""; }

int osg_match_last_stats(osg_ctx *ctx, int32_t *out4)
{
    if (!ctx || !out4) return OSG_E_INVALID;
    for (int i = 0; i < 4; i++) out4[i] = ctx->match_stats[i];
    return OSG_OK;
}

int osg_ctx_last_kernel_ms(osg_ctx *ctx, double *ms)
{
    if (!ctx || !ms) return OSG_E_INVALID;
    *ms = ctx->last_kernel_ms;
    return OSG_OK;
}

int osg_ctx_device_bytes(osg_ctx *ctx, int64_t *bytes)
{
    if (!ctx || !bytes) return OSG_E_INVALID;
    int64_t t = 0;
    for (int s = 0; s < SLOT_COUNT; s++) t += (int64_t)ctx->cap[s];
    *bytes = t;
    return OSG_OK;
}

// ref:src/ORBmatcher.cc:2388-2408 — host scalar form (the SWAR popcount as written).
int osg_descriptor_distance(const uint8_t *a, const uint8_t *b)
{
    if (!a || !b) return OSG_E_INVALID;
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        int32_t wa, wb;
        std::memcpy(&wa, a + 4 * i, 4);
        std::memcpy(&wb, b + 4 * i, 4);
        unsigned int v = (unsigned int)(wa ^ wb);
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}

}  // extern "C"
