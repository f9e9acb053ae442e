// Multi-GPU reduction of PseudoAlignment counters over RCCL (xGMI), part of the
// C ABI (include/pa.h).  SURVEY.md section 8(b)/(e): reads shard across the
// GPUs of a node with no exchange on the data path; a job ends with ONE
// all-reduce of each pa_result's two device blocks,
//   sum block [6 stats | G unique | G ambiguous]  -> ncclSum  (uint64)
//   min block [G first-appearance keys]           -> ncclMin  (uint64)
// (16 G + 48 bytes: latency-bound, one call each).  Because the first keys
// carry GLOBAL read indices, the reduced blocks order the Summary exactly as one
// process walking all reads would (src/kmer.py:639-657, quirk 9).
//
// RCCL is opened at the first call (dlopen "librccl.so.1", or PA_RCCL_LIBRARY),
// not linked: libpa.so loads on hosts without it, and in a process where torch
// already loaded its RCCL the loader returns that same library (one SONAME),
// so a communicator made by either can be used with the other's calls.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "pa_internal.h"

namespace {

// The subset of rccl.h used here (ABI-stable NCCL 2.x types).
typedef struct ncclComm *ncclComm_t;
typedef struct {
    char internal[128];
} ncclUniqueId;
typedef int ncclResult_t;      // ncclSuccess = 0
enum { kNcclUint64 = 5 };      // ncclDataType_t ncclUint64
enum { kNcclSum = 0, kNcclMin = 3 };  // ncclRedOp_t

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_count)(const ncclComm_t, int *) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    std::string err;
    bool ok = false;
};

Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // RCCL from the ROCm whose HIP runtime this process runs libpa.so on
        // (the directory of the libamdhip64 that hipGetDeviceCount resolved
        // to): a process that also maps torch's bundled runtime otherwise may
        // get an RCCL of the other runtime, which sees no device
        // ("pfn_hsa_system_get_info failed", round 6)
        const char *path = std::getenv("PA_RCCL_LIBRARY");
        void *h = nullptr;
        if (path && *path) {
            h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
        } else {
            Dl_info info{};
            if (dladdr((void *)&hipGetDeviceCount, &info) && info.dli_fname) {
                std::string dir(info.dli_fname);
                const size_t cut = dir.rfind('/');
                if (cut != std::string::npos) {
                    dir.resize(cut);
                    for (const char *name : {"/librccl.so.1", "/librccl.so"})
                        if (!h) h = dlopen((dir + name).c_str(), RTLD_NOW | RTLD_LOCAL);
                }
            }
            if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        }
        if (!h) {
            r.err = std::string("RCCL not available: ") + dlerror();
            return;
        }
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
        r.comm_count = (decltype(r.comm_count))dlsym(h, "ncclCommCount");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.comm_count;
        if (!r.ok) r.err = "RCCL library lacks an expected symbol";
    });
    return r;
}

pa_status rccl_status(ncclResult_t e, const char *what) {
    if (e == 0) return PA_OK;
    const Rccl &r = rccl();
    pa::set_error(std::string(what) + ": " + (r.error_string ? r.error_string(e) : std::to_string(e)));
    return PA_EDEVICE;
}

}  // namespace

#define PA_NEED_RCCL()                      \
    do {                                    \
        if (!rccl().ok) {                   \
            pa::set_error(rccl().err);      \
            return PA_EUNSUPPORTED;         \
        }                                   \
    } while (0)

extern "C" {

pa_status pa_comm_unique_id(uint8_t *id) {
    if (!id) {
        pa::set_error("id must not be NULL");
        return PA_EINVAL;
    }
    PA_NEED_RCCL();
    ncclUniqueId u;
    PA_TRY(rccl_status(rccl().get_unique_id(&u), "ncclGetUniqueId"));
    std::memcpy(id, u.internal, PA_COMM_ID_BYTES);
    return PA_OK;
}

pa_status pa_comm_init(int32_t device, int32_t nranks, int32_t rank, const uint8_t *id, void **comm) {
    if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) {
        pa::set_error("pa_comm_init: bad arguments (need 0 <= rank < nranks, id and comm not NULL)");
        return PA_EINVAL;
    }
    *comm = nullptr;
    PA_NEED_RCCL();
    PA_HIP(hipSetDevice(device));
    ncclUniqueId u;
    std::memcpy(u.internal, id, PA_COMM_ID_BYTES);
    ncclComm_t c = nullptr;
    PA_TRY(rccl_status(rccl().comm_init_rank(&c, nranks, u, rank), "ncclCommInitRank"));
    *comm = c;
    return PA_OK;
}

pa_status pa_comm_free(void *comm) {
    if (!comm) return PA_OK;
    PA_NEED_RCCL();
    return rccl_status(rccl().comm_destroy((ncclComm_t)comm), "ncclCommDestroy");
}

pa_status pa_comm_count(void *comm, int32_t *nranks) {
    if (!comm || !nranks) {
        pa::set_error("pa_comm_count: comm and nranks must not be NULL");
        return PA_EINVAL;
    }
    PA_NEED_RCCL();
    int n = 0;
    PA_TRY(rccl_status(rccl().comm_count((ncclComm_t)comm, &n), "ncclCommCount"));
    *nranks = n;
    return PA_OK;
}

pa_status pa_counters_reduce(pa_result *res, void *comm, void *stream) {
    if (!res || !comm) {
        pa::set_error("pa_counters_reduce: res and comm must not be NULL");
        return PA_EINVAL;
    }
    PA_NEED_RCCL();
    PA_HIP(hipSetDevice(res->device));
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const uint64_t G = res->n_genomes;
    // counts and keys are < 2^63, so the unsigned SUM / MIN are exact
    PA_TRY(rccl_status(rccl().all_reduce(res->sum_block, res->sum_block, 6 + 2 * G, kNcclUint64, kNcclSum,
                                         (ncclComm_t)comm, st),
                       "ncclAllReduce(sum block)"));
    if (G) {
        PA_TRY(rccl_status(rccl().all_reduce(res->min_block, res->min_block, G, kNcclUint64, kNcclMin,
                                             (ncclComm_t)comm, st),
                           "ncclAllReduce(min block)"));
    }
    return PA_OK;
}

}  // extern "C"
