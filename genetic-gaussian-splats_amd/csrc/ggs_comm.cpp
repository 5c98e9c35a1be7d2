// Multi-GPU fitness gather over RCCL: candidates are sharded
// across the GPUs of a node, one process per GPU, and the only exchange is an
// all-gather of every rank's fitness scalars (xGMI).  The reference is
// single-device (render.py:4, fitness.py:34-47 evaluates one list on one GPU);
// this is the collective its sharded evaluation needs.
//
// The gather is enqueued by the library on the caller's stream (in order after
// the fitness kernels) or on the communicator's own stream (overlap: the next
// batch's raster runs while the scalars move).  RCCL is loaded at first use:
// the copy already in the process when there is one (ggs/_lib.py preload_rccl
// loads the one beside the HIP runtime, RTLD_LOCAL), else $GGS_RCCL, else
// librccl.so.1 / librccl.so from the directory of the HIP runtime libggs is
// bound to (by absolute path, never a search).  It must come from that same
// directory (one ROCm tree: /opt/rocm's, or PyTorch's bundled copies): a mixed
// pair is refused, because HIP and RCCL of different ROCm releases in one
// process fail at the first N > 1 communicator (docs/EXPERIMENTS.md §16).
#include <dlfcn.h>
#include <limits.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types and enums only; entry points are resolved by dlsym
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ggs.h"

namespace ggs {
int set_error(int code, const char* msg);   // ggs_capi.cpp (thread-local ggs_last_error)
namespace {

int cfail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return set_error(code, buf);
}

struct Rccl {
    ncclResult_t (*get_version)(int*) = nullptr;
    ncclResult_t (*comm_count)(ncclComm_t, int*) = nullptr;
    ncclResult_t (*comm_user_rank)(ncclComm_t, int*) = nullptr;
    ncclResult_t (*comm_cu_device)(ncclComm_t, int*) = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    std::string err;
    std::string path;                    // the loaded library (realpath), "" before / on failure
    int version = 0;
    bool ok = false;
};

// realpath of the shared object holding `sym` ("" if unknown)
std::string object_path(const void* sym) {
    Dl_info info{};
    if (!sym || !dladdr(sym, &info) || !info.dli_fname) return "";
    char buf[PATH_MAX];
    return realpath(info.dli_fname, buf) ? std::string(buf) : std::string(info.dli_fname);
}
std::string dir_of(const std::string& p) {
    const size_t k = p.rfind('/');
    return k == std::string::npos ? std::string(".") : p.substr(0, k);
}
// the HIP runtime libggs is bound to
std::string hip_runtime_path() { return object_path(reinterpret_cast<const void*>(&hipGetDevice)); }

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const std::string hip = hip_runtime_path(), hdir = dir_of(hip);
        // RTLD_LOCAL: RCCL's exported libstdc++ template instantiations must not
        // enter the global scope (PyTorch's bundled librccl, loaded RTLD_GLOBAL
        // before torch, had torch's libraries bind their std::map / shared_ptr
        // code to its copies: "double free or corruption" at exit, EXP §16)
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h && getenv("GGS_RCCL")) h = dlopen(getenv("GGS_RCCL"), RTLD_NOW | RTLD_LOCAL);
        for (const char* name : {"/librccl.so.1", "/librccl.so"})
            if (!h && !hip.empty()) h = dlopen((hdir + name).c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            r.err = std::string("cannot load RCCL beside the HIP runtime (") + hdir + "): " + (e ? e : "?");
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
        r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
        r.get_version = (decltype(r.get_version))dlsym(h, "ncclGetVersion");
        r.comm_count = (decltype(r.comm_count))dlsym(h, "ncclCommCount");
        r.comm_user_rank = (decltype(r.comm_user_rank))dlsym(h, "ncclCommUserRank");
        r.comm_cu_device = (decltype(r.comm_cu_device))dlsym(h, "ncclCommCuDevice");
        r.ok = r.get_unique_id && r.comm_init_rank && r.all_gather && r.comm_destroy && r.error_string &&
               r.comm_init_all && r.group_start && r.group_end && r.get_version && r.comm_count &&
               r.comm_user_rank && r.comm_cu_device;
        if (!r.ok) {
            r.err = "RCCL is missing an entry point (ncclGetUniqueId / ncclCommInitRank / ncclCommInitAll / "
                    "ncclAllGather / ncclGroupStart / ncclGroupEnd / ncclCommDestroy / ncclGetErrorString / "
                    "ncclGetVersion / ncclCommCount / ncclCommUserRank / ncclCommCuDevice)";
            return;
        }
        r.path = object_path(reinterpret_cast<const void*>(r.get_unique_id));
        if (r.get_version(&r.version) != ncclSuccess) r.version = 0;
        // one ROCm tree: RCCL from the HIP runtime's directory
        if (hip.empty() || dir_of(r.path) != hdir) {
            r.ok = false;
            r.err = "RCCL " + r.path + " is not from the HIP runtime's tree (" + (hip.empty() ? "?" : hip) +
                    "): refusing a process that mixes ROCm trees (load RCCL beside the HIP runtime: "
                    "ggs._lib.preload_rccl)";
        }
    });
    return r;
}

#define GGS_NCCL(call)                                                                           \
    do {                                                                                         \
        ncclResult_t r_ = (call);                                                                \
        if (r_ != ncclSuccess)                                                                   \
            return cfail(GGS_EHIP, "%s: %s", #call, R.error_string(r_));                         \
    } while (0)
#define GGS_HIPC(call)                                                                           \
    do {                                                                                         \
        hipError_t e_ = (call);                                                                  \
        if (e_ != hipSuccess) return cfail(GGS_EHIP, "%s: %s", #call, hipGetErrorString(e_));    \
    } while (0)

constexpr int kTickets = 64;   // gathers a caller may still wait on

struct Comm {
    int dev = 0, nranks = 1, rank = 0;
    ncclComm_t nc = nullptr;
    hipStream_t side = nullptr;          // overlap mode: gathers run here
    hipEvent_t ready = nullptr;          // caller's stream -> side
    hipEvent_t done[kTickets] = {};      // side -> caller's stream, one per ticket slot
    int64_t issued = 0;                  // tickets handed out
    float* scratch = nullptr;            // barrier / host all-gather staging (device)
    int64_t scratch_cap = 0;             // floats
    std::mutex mu;
    std::shared_ptr<struct Loop> loop;   // loopback group (ggs_comm_init_loopback), no RCCL
};

// Loopback group: n communicators on ONE device in one process that act as
// ranks 0..n-1 of one job, so the sharded paths (rank != 0, uneven and empty
// shards, the fingerprint exchange) run on a one-GPU box.  Device all-gathers
// are matched by sequence number: each rank's call records an event after the
// work already on its stream (the producer of its send buffer) and returns;
// the LAST rank's call enqueues, on every rank's stream, the waits on the
// others' events and the device-to-device copies of their shards, then joins
// the streams again (every stream waits for every copy), so no rank's later
// work rewrites a shard another rank has still to read.  A rank that calls
// again before every rank called fails (loopback ranks run in lockstep).
// Host all-gathers are a blocking rendezvous (ranks on separate host threads),
// bounded by GGS_LOOPBACK_TIMEOUT_S (default 60 s): a missing rank fails loudly.
struct Loop {
    int n = 1, dev = 0;
    std::mutex mu;
    std::condition_variable cv;
    // device gathers
    int64_t seq = 0;                     // the gather being collected
    int arrived = 0;
    std::vector<char> have;
    std::vector<hipStream_t> st;
    std::vector<const float*> send;
    std::vector<float*> recv;
    std::vector<int64_t> count;
    std::vector<hipEvent_t> ev, done;
    std::string broken;                  // set when an enqueue failed part-way: the group is unusable
    // host gathers
    int64_t hgen = 0;
    int harrived = 0;
    int64_t hcount = -1;
    std::vector<float> hbuf, hres;
    ~Loop() {
        for (auto e : ev) if (e) (void)hipEventDestroy(e);
        for (auto e : done) if (e) (void)hipEventDestroy(e);
    }
};

// Staging for the host-pointer collectives: [count | nranks*count] floats.
int ensure_scratch(Comm* c, int64_t floats) {
    if (floats <= c->scratch_cap) return GGS_OK;
    if (c->scratch) (void)hipFree(c->scratch);
    c->scratch = nullptr;
    c->scratch_cap = 0;
    const int64_t want = std::max<int64_t>(floats, 1024);
    GGS_HIPC(hipMalloc((void**)&c->scratch, sizeof(float) * (size_t)want));
    c->scratch_cap = want;
    return GGS_OK;
}

// The communicator's own stream and its events, made at the first call that
// needs them (an overlapped gather or a host-side collective): a communicator
// used only for in-stream gathers holds no stream of its own, so it takes no
// hardware queue (bench.py counts the streams that carry collectives against
// GPU_MAX_HW_QUEUES).  Called with c->mu held and c->dev current.
int ensure_side(Comm* c) {
    if (c->side) return GGS_OK;
    hipStream_t s = nullptr;
    hipError_t he = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (he == hipSuccess && !c->ready) he = hipEventCreateWithFlags(&c->ready, hipEventDisableTiming);
    for (int i = 0; he == hipSuccess && i < kTickets; ++i)
        if (!c->done[i]) he = hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming);
    if (he != hipSuccess) {
        if (s) (void)hipStreamDestroy(s);
        return cfail(GGS_EHIP, "communicator stream set-up: %s", hipGetErrorString(he));
    }
    c->side = s;
    return GGS_OK;
}

// A gather over one rank is a copy: done by a small kernel on the stream, not
// through RCCL (whose single-rank path costs a stream-ordering round trip).
__global__ void __launch_bounds__(256) copy_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                   int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

struct DevScope {
    int prev = -1;
    explicit DevScope(int d) { if (hipGetDevice(&prev) != hipSuccess) prev = -1; (void)hipSetDevice(d); }
    ~DevScope() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// d_recv on rank r's stream is defined only once EVERY rank has called for this
// gather: the last caller enqueues all the copies (ranks must be stepped in
// lockstep; include/ggs.h).  A HIP failure part-way through that enqueue leaves
// some streams with copies and others without, so the group is poisoned: every
// later call fails with the first error instead of pairing the wrong gathers.
int loop_allgather(Comm* c, hipStream_t stream, const float* d_send, float* d_recv, int64_t count) {
    Loop& L = *c->loop;
    std::lock_guard<std::mutex> lk(L.mu);
    if (!L.broken.empty())
        return cfail(GGS_EHIP, "loopback group unusable after an earlier failure: %s", L.broken.c_str());
    const int r = c->rank;
    if (L.have[r])
        return cfail(GGS_EINVAL, "loopback all-gather %lld: rank %d called again before every rank called "
                     "(loopback ranks must be stepped in lockstep)", (long long)L.seq, r);
    if (L.arrived > 0 && count != L.count[std::find(L.have.begin(), L.have.end(), 1) - L.have.begin()])
        return cfail(GGS_EINVAL, "loopback all-gather %lld: rank %d sends %lld floats, another rank a different "
                     "count", (long long)L.seq, r, (long long)count);
    DevScope ds(L.dev);
    GGS_HIPC(hipEventRecord(L.ev[r], stream));
    L.have[r] = 1;
    L.st[r] = stream;
    L.send[r] = d_send;
    L.recv[r] = d_recv;
    L.count[r] = count;
    if (++L.arrived < L.n) return GGS_OK;
    const size_t bytes = sizeof(float) * (size_t)count;
    hipError_t e = hipSuccess;
    const char* what = "";
    for (int q = 0; q < L.n && e == hipSuccess; ++q) {               // rank q's stream receives every shard
        for (int p = 0; p < L.n && e == hipSuccess; ++p) {
            float* dst = L.recv[q] + (int64_t)p * count;
            if (p != q && (e = hipStreamWaitEvent(L.st[q], L.ev[p], 0)) != hipSuccess) what = "hipStreamWaitEvent";
            else if (bytes && dst != L.send[p] &&
                     (e = hipMemcpyAsync(dst, L.send[p], bytes, hipMemcpyDeviceToDevice, L.st[q])) != hipSuccess)
                what = "hipMemcpyAsync";
        }
        if (e == hipSuccess && (e = hipEventRecord(L.done[q], L.st[q])) != hipSuccess) what = "hipEventRecord";
    }
    for (int q = 0; q < L.n && e == hipSuccess; ++q)
        for (int p = 0; p < L.n && e == hipSuccess; ++p)
            if (p != q && (e = hipStreamWaitEvent(L.st[q], L.done[p], 0)) != hipSuccess) what = "hipStreamWaitEvent";
    std::fill(L.have.begin(), L.have.end(), 0);
    L.arrived = 0;
    ++L.seq;
    if (e != hipSuccess) {
        char m[256];
        snprintf(m, sizeof m, "gather %lld: %s: %s", (long long)(L.seq - 1), what, hipGetErrorString(e));
        L.broken = m;
        return cfail(GGS_EHIP, "loopback all-gather failed part-way (%s); the group is now unusable", m);
    }
    return GGS_OK;
}

int loop_allgather_host(Comm* c, const float* send, float* recv, int64_t count) {
    Loop& L = *c->loop;
    std::unique_lock<std::mutex> lk(L.mu);
    if (L.harrived == 0) {
        L.hcount = count;
        L.hbuf.assign((size_t)L.n * (size_t)std::max<int64_t>(count, 0), 0.0f);
    } else if (count != L.hcount) {
        return cfail(GGS_EINVAL, "loopback host all-gather: rank %d sends %lld floats, rank(s) before it %lld",
                     c->rank, (long long)count, (long long)L.hcount);
    }
    if (count > 0) memcpy(L.hbuf.data() + (int64_t)c->rank * count, send, sizeof(float) * (size_t)count);
    const int64_t gen = L.hgen;
    if (++L.harrived == L.n) {
        L.hres.swap(L.hbuf);
        L.harrived = 0;
        ++L.hgen;
        L.cv.notify_all();
    } else {
        const char* t = getenv("GGS_LOOPBACK_TIMEOUT_S");
        const double secs = t ? atof(t) : 60.0;
        if (!L.cv.wait_for(lk, std::chrono::duration<double>(secs), [&] { return L.hgen != gen; })) {
            --L.harrived;
            return cfail(GGS_EHIP, "loopback host all-gather: rank %d waited %.0f s for the other %d rank(s) "
                         "(each loopback rank needs its own host thread)", c->rank, secs, L.n - L.harrived - 1);
        }
    }
    if (count > 0) memcpy(recv, L.hres.data(), sizeof(float) * (size_t)count * L.n);
    return GGS_OK;
}

}  // namespace
}  // namespace ggs

using namespace ggs;

extern "C" {

int ggs_comm_unique_id(uint8_t* id128) {
    const Rccl& R = rccl();
    if (!R.ok) return cfail(GGS_ENODEV, "%s", R.err.c_str());
    if (!id128) return cfail(GGS_EINVAL, "ggs_comm_unique_id: null output");
    static_assert(sizeof(ncclUniqueId) == GGS_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    GGS_NCCL(R.get_unique_id(&u));
    memcpy(id128, &u, sizeof u);
    return GGS_OK;
}

int ggs_comm_create(int32_t device, int32_t nranks, int32_t rank, const uint8_t* id128, void** comm) {
    const Rccl& R = rccl();
    if (!R.ok) return cfail(GGS_ENODEV, "%s", R.err.c_str());
    if (!comm || !id128 || nranks < 1 || rank < 0 || rank >= nranks)
        return cfail(GGS_EINVAL, "ggs_comm_create: need 0 <= rank (%d) < nranks (%d), id and comm", rank, nranks);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return cfail(GGS_ENODEV, "ggs_comm_create: device %d not available (%d visible)", device, ndev);
    DevScope ds(device);
    Comm* c = new Comm;
    c->dev = device;
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId u;
    memcpy(&u, id128, sizeof u);
    int rc = GGS_OK;
    ncclResult_t nr = R.comm_init_rank(&c->nc, nranks, u, rank);
    if (nr != ncclSuccess) rc = cfail(GGS_EHIP, "ncclCommInitRank: %s", R.error_string(nr));
    if (rc) {
        ggs_comm_destroy(c);
        return rc;
    }
    *comm = c;
    return GGS_OK;
}

int ggs_comm_allgather(void* comm, void* stream, const float* d_send, float* d_recv, int64_t count,
                       int32_t overlap, int64_t* ticket) {
    Comm* c = (Comm*)comm;
    if (c && c->loop) {
        if (count < 0 || (count > 0 && (!d_send || !d_recv)))
            return cfail(GGS_EINVAL, "ggs_comm_allgather: count %lld with null buffers", (long long)count);
        if (overlap) return cfail(GGS_EINVAL, "ggs_comm_allgather: a loopback communicator gathers in-stream only");
        if (ticket) *ticket = -1;
        return loop_allgather(c, (hipStream_t)stream, d_send, d_recv, count);
    }
    const Rccl& R = rccl();
    if (!c || !R.ok) return cfail(GGS_EINVAL, "ggs_comm_allgather: no communicator");
    if (count < 0 || (count > 0 && (!d_send || !d_recv)))
        return cfail(GGS_EINVAL, "ggs_comm_allgather: count %lld with null buffers", (long long)count);
    std::lock_guard<std::mutex> lk(c->mu);
    DevScope ds(c->dev);
    hipStream_t st = (hipStream_t)stream;
    if (c->nranks == 1 && !overlap && !getenv("GGS_COMM_RCCL_SELF")) {
        if (count > 0 && d_send != d_recv) {
            const unsigned grid = (unsigned)std::min<int64_t>((count + 255) / 256, 1024);
            hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, st, d_send, d_recv, count);
            GGS_HIPC(hipGetLastError());
        }
        if (ticket) *ticket = -1;
        return GGS_OK;
    }
    if (!overlap) {
        GGS_NCCL(R.all_gather(d_send, d_recv, (size_t)count, ncclFloat32, c->nc, st));
        if (ticket) *ticket = -1;
        return GGS_OK;
    }
    // overlap: the gather waits for the work already on `stream` (the fitness
    // kernels that wrote d_send), then runs on the side stream
    if (int rc = ensure_side(c)) return rc;
    GGS_HIPC(hipEventRecord(c->ready, st));
    GGS_HIPC(hipStreamWaitEvent(c->side, c->ready, 0));
    GGS_NCCL(R.all_gather(d_send, d_recv, (size_t)count, ncclFloat32, c->nc, c->side));
    const int64_t t = c->issued++;
    GGS_HIPC(hipEventRecord(c->done[t % kTickets], c->side));
    if (ticket) *ticket = t;
    return GGS_OK;
}

int ggs_comm_wait(void* comm, void* stream, int64_t ticket) {
    Comm* c = (Comm*)comm;
    if (!c) return cfail(GGS_EINVAL, "ggs_comm_wait: no communicator");
    std::lock_guard<std::mutex> lk(c->mu);
    if (ticket < 0) return GGS_OK;                       // in-stream gather: nothing to join
    if (ticket >= c->issued) return cfail(GGS_EINVAL, "ggs_comm_wait: ticket %lld not issued", (long long)ticket);
    DevScope ds(c->dev);
    // a slot reused by a later ticket still orders after `ticket` (one side stream)
    GGS_HIPC(hipStreamWaitEvent((hipStream_t)stream, c->done[ticket % kTickets], 0));
    return GGS_OK;
}

int ggs_comm_info(void* comm, int32_t* nranks, int32_t* rank, int32_t* device) {
    Comm* c = (Comm*)comm;
    if (!c) return cfail(GGS_EINVAL, "ggs_comm_info: no communicator");
    if (c->loop || !c->nc) return cfail(GGS_EINVAL, "ggs_comm_info: not an RCCL communicator (loopback group)");
    const Rccl& R = rccl();
    if (!R.ok) return cfail(GGS_ENODEV, "%s", R.err.c_str());
    int n = 0, r = 0, d = 0;
    GGS_NCCL(R.comm_count(c->nc, &n));
    GGS_NCCL(R.comm_user_rank(c->nc, &r));
    GGS_NCCL(R.comm_cu_device(c->nc, &d));
    if (nranks) *nranks = n;
    if (rank) *rank = r;
    if (device) *device = d;
    return GGS_OK;
}

int ggs_runtime_info(char* buf, int32_t cap) {
    // RCCL as loaded by this library (not loaded by this call: null until a
    // communicator or ggs_comm_unique_id needed it)
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    const std::string hip = hip_runtime_path();
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    std::string rpath;
    int ver = 0;
    if (h) {
        void* f = dlsym(h, "ncclGetUniqueId");
        rpath = object_path(f);
        auto gv = (ncclResult_t(*)(int*))dlsym(h, "ncclGetVersion");
        if (!gv || gv(&ver) != ncclSuccess) ver = 0;
        dlclose(h);
    }
    int hv = 0;
    if (hipRuntimeGetVersion(&hv) != hipSuccess) hv = 0;
    auto q = [](const std::string& x) { return x.empty() ? std::string("null") : "\"" + x + "\""; };
    std::string j = "{\"hip\": " + q(hip) + ", \"hip_version\": " + std::to_string(hv) + ", \"rccl\": " + q(rpath) +
                    ", \"rccl_version\": " + (rpath.empty() ? std::string("null") : std::to_string(ver)) +
                    ", \"same_tree\": " +
                    (rpath.empty() || hip.empty() ? std::string("null")
                                                  : std::string(dir_of(rpath) == dir_of(hip) ? "true" : "false")) +
                    "}";
    if (!buf || cap <= (int32_t)j.size()) return (int32_t)j.size() + 1;     // the size needed
    memcpy(buf, j.c_str(), j.size() + 1);
    return GGS_OK;
}

int ggs_comm_size(void* comm, int32_t* nranks, int32_t* rank) {
    Comm* c = (Comm*)comm;
    if (!c) return cfail(GGS_EINVAL, "ggs_comm_size: no communicator");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return GGS_OK;
}

void ggs_comm_destroy(void* comm) {
    Comm* c = (Comm*)comm;
    if (!c) return;
    {
        DevScope ds(c->dev);
        if (c->side) (void)hipStreamSynchronize(c->side);
        if (c->nc) {
            const Rccl& R = rccl();
            if (R.ok) (void)R.comm_destroy(c->nc);
        }
        for (int i = 0; i < kTickets; ++i)
            if (c->done[i]) (void)hipEventDestroy(c->done[i]);
        if (c->ready) (void)hipEventDestroy(c->ready);
        if (c->side) (void)hipStreamDestroy(c->side);
        if (c->scratch) (void)hipFree(c->scratch);
    }
    delete c;
}

int ggs_comm_init_local(int32_t n, const int32_t* devices, void** comms) {
    const Rccl& R = rccl();
    if (!R.ok) return cfail(GGS_ENODEV, "%s", R.err.c_str());
    if (n < 1 || !devices || !comms) return cfail(GGS_EINVAL, "ggs_comm_init_local: need n >= 1 devices and outputs");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    for (int i = 0; i < n; ++i) {
        if (devices[i] < 0 || devices[i] >= ndev)
            return cfail(GGS_ENODEV, "ggs_comm_init_local: device %d not available (%d visible)", devices[i], ndev);
        for (int j = 0; j < i; ++j)
            if (devices[j] == devices[i]) return cfail(GGS_EINVAL, "ggs_comm_init_local: device %d listed twice", devices[i]);
    }
    std::vector<ncclComm_t> ncs(n, nullptr);
    {
        ncclResult_t nr = R.comm_init_all(ncs.data(), n, devices);
        if (nr != ncclSuccess) return cfail(GGS_EHIP, "ncclCommInitAll: %s", R.error_string(nr));
    }
    for (int i = 0; i < n; ++i) {
        Comm* c = new Comm;
        c->dev = devices[i];
        c->nranks = n;
        c->rank = i;
        c->nc = ncs[i];
        comms[i] = c;
    }
    return GGS_OK;
}

int ggs_comm_allgather_host(void* comm, const float* send, float* recv, int64_t count) {
    Comm* c = (Comm*)comm;
    if (count < 0 || (count > 0 && (!send || !recv)))
        return cfail(GGS_EINVAL, "ggs_comm_allgather_host: count %lld with null buffers", (long long)count);
    if (c && c->loop) return loop_allgather_host(c, send, recv, count);
    const Rccl& R = rccl();
    if (!c || !R.ok) return cfail(GGS_EINVAL, "ggs_comm_allgather_host: no communicator");
    std::lock_guard<std::mutex> lk(c->mu);
    DevScope ds(c->dev);
    const int64_t cnt = std::max<int64_t>(count, 1);    // a zero-length call still synchronises the ranks
    int rc = ensure_side(c);
    if (!rc) rc = ensure_scratch(c, cnt * (1 + c->nranks));
    if (rc) return rc;
    float* d_send = c->scratch;
    float* d_recv = c->scratch + cnt;
    if (count > 0)
        GGS_HIPC(hipMemcpyAsync(d_send, send, sizeof(float) * (size_t)count, hipMemcpyHostToDevice, c->side));
    else
        GGS_HIPC(hipMemsetAsync(d_send, 0, sizeof(float), c->side));
    GGS_NCCL(R.all_gather(d_send, d_recv, (size_t)cnt, ncclFloat32, c->nc, c->side));
    if (count > 0) {
        for (int r = 0; r < c->nranks; ++r)
            GGS_HIPC(hipMemcpyAsync(recv + (int64_t)r * count, d_recv + (int64_t)r * cnt, sizeof(float) * (size_t)count,
                                    hipMemcpyDeviceToHost, c->side));
    }
    GGS_HIPC(hipStreamSynchronize(c->side));
    return GGS_OK;
}

int ggs_comm_barrier(void* comm) { return ggs_comm_allgather_host(comm, nullptr, nullptr, 0); }

int ggs_comm_init_loopback(int32_t device, int32_t n, void** comms) {
    if (n < 1 || !comms) return cfail(GGS_EINVAL, "ggs_comm_init_loopback: need n >= 1 and outputs");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return cfail(GGS_ENODEV, "ggs_comm_init_loopback: device %d not available (%d visible)", device, ndev);
    DevScope ds(device);
    auto L = std::make_shared<Loop>();
    L->n = n;
    L->dev = device;
    L->have.assign(n, 0);
    L->st.assign(n, nullptr);
    L->send.assign(n, nullptr);
    L->recv.assign(n, nullptr);
    L->count.assign(n, 0);
    L->ev.assign(n, nullptr);
    L->done.assign(n, nullptr);
    for (int i = 0; i < n; ++i) {
        GGS_HIPC(hipEventCreateWithFlags(&L->ev[i], hipEventDisableTiming));
        GGS_HIPC(hipEventCreateWithFlags(&L->done[i], hipEventDisableTiming));
    }
    for (int i = 0; i < n; ++i) {
        Comm* c = new Comm;
        c->dev = device;
        c->nranks = n;
        c->rank = i;
        c->loop = L;
        comms[i] = c;
    }
    return GGS_OK;
}

}  // extern "C"

namespace ggs {
// Single-process fan-out (ggs_capi.cpp): one in-place all-gather per device of
// that device's `per`-float shard of buf[d] (shard d at buf[d] + d*per), grouped
// so one thread can drive every device.
int comm_group_allgather_inplace(void* const* comms, int n, hipStream_t const* streams, float* const* bufs,
                                 int64_t per) {
    const Rccl& R = rccl();
    if (!R.ok) return cfail(GGS_ENODEV, "%s", R.err.c_str());
    GGS_NCCL(R.group_start());
    ncclResult_t first_err = ncclSuccess;
    for (int d = 0; d < n; ++d) {
        Comm* c = (Comm*)comms[d];
        DevScope ds(c->dev);
        ncclResult_t r = R.all_gather(bufs[d] + (int64_t)c->rank * per, bufs[d], (size_t)per, ncclFloat32, c->nc,
                                      streams[d]);
        if (r != ncclSuccess && first_err == ncclSuccess) first_err = r;
    }
    GGS_NCCL(R.group_end());
    if (first_err != ncclSuccess) return cfail(GGS_EHIP, "ncclAllGather: %s", R.error_string(first_err));
    return GGS_OK;
}
}  // namespace ggs
