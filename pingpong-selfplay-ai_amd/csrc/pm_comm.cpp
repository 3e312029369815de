// The learner's exchange step without a framework in the loop: an RCCL communicator owned by the
// library, and the sharded vector steps issued from C with the gradient all-reduce enqueued on the
// SAME stream as the kernels around it.
//
// Through torch.distributed every all-reduce crosses to the process group's internal stream and back
// (an event record + wait each way) and costs a Python call; here a vector step of a sharded learner
// is one library call: k_actenv, k_learn (+ next step's side-A act), ncclAllReduce(sp->grad),
// k_adam, all in stream order. Bit-identical to the Python sequence with torch's all_reduce (the same
// RCCL sum of the same buffer).
//
// RCCL is bound at run time (dlopen of the caller-supplied library path: the process's own RCCL —
// torch's bundled librccl.so when torch has loaded it — so one RCCL instance serves both), so
// libpongmi does not link it and loads without it.
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

#include "pm_host.h"

namespace {

// The subset of rccl.h used here (ABI of NCCL 2.x / RCCL: opaque 128-byte id, int enums).
typedef struct ncclComm* ncclComm_t;
typedef struct {
    char internal[PM_COMM_ID_BYTES];
} ncclUniqueId;
typedef int ncclResult_t;
constexpr int kNcclFloat32 = 7;
constexpr int kNcclSum = 0;

struct Rccl {
    void* handle = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*comm_user_rank)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*comm_device)(const ncclComm_t, int*) = nullptr;
};

int bind(const char* path, Rccl& r) {
    PM_REQUIRE(path && *path, PM_E_ARG, "pm_comm: empty RCCL library path");
    void* h = dlopen(path, RTLD_NOW | RTLD_NOLOAD);  // the instance the process already runs, if any
    if (!h) h = dlopen(path, RTLD_NOW);
    PM_REQUIRE(h, PM_E_COMM, "pm_comm: dlopen(%s): %s", path, dlerror());
    r.handle = h;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.comm_count = (decltype(r.comm_count))dlsym(h, "ncclCommCount");
    r.comm_user_rank = (decltype(r.comm_user_rank))dlsym(h, "ncclCommUserRank");
    r.comm_device = (decltype(r.comm_device))dlsym(h, "ncclCommCuDevice");
    PM_REQUIRE(r.get_unique_id && r.comm_init_rank && r.all_reduce && r.comm_destroy && r.error_string, PM_E_COMM,
               "pm_comm: %s lacks the ncclGetUniqueId / ncclCommInitRank / ncclAllReduce / ncclCommDestroy / "
               "ncclGetErrorString symbols",
               path);
    return PM_OK;
}

}  // namespace

struct pm_comm {
    Rccl rccl;
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0;
};

extern "C" int pm_comm_unique_id(const char* rccl_path, uint8_t* id) {
    PM_REQUIRE(id, PM_E_ARG, "pm_comm_unique_id: null id");
    Rccl r;
    int rc = bind(rccl_path, r);
    if (rc) return rc;
    ncclUniqueId u;
    const ncclResult_t e = r.get_unique_id(&u);
    PM_REQUIRE(e == 0, PM_E_COMM, "ncclGetUniqueId: %s", r.error_string(e));
    memcpy(id, u.internal, PM_COMM_ID_BYTES);
    return PM_OK;
}

extern "C" int pm_comm_init(const char* rccl_path, const uint8_t* id, int32_t nranks, int32_t rank, pm_comm** out) {
    PM_REQUIRE(id && out, PM_E_ARG, "pm_comm_init: null id / out");
    PM_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, PM_E_ARG, "pm_comm_init: rank %d of %d", rank, nranks);
    *out = nullptr;
    pm_comm* c = new pm_comm();
    int rc = bind(rccl_path, c->rccl);
    if (rc) {
        delete c;
        return rc;
    }
    ncclUniqueId u;
    memcpy(u.internal, id, PM_COMM_ID_BYTES);
    const ncclResult_t e = c->rccl.comm_init_rank(&c->comm, nranks, u, rank);  // collective over the ranks
    if (e != 0) {
        const char* msg = c->rccl.error_string(e);
        delete c;
        return pm_fail(PM_E_COMM, "ncclCommInitRank(rank %d of %d): %s", rank, nranks, msg);
    }
    c->nranks = nranks;
    c->rank = rank;
    *out = c;
    return PM_OK;
}

extern "C" int pm_comm_destroy(pm_comm* c) {
    if (!c) return PM_OK;
    const ncclResult_t e = c->comm ? c->rccl.comm_destroy(c->comm) : 0;
    const char* msg = e ? c->rccl.error_string(e) : "";
    delete c;
    PM_REQUIRE(e == 0, PM_E_COMM, "ncclCommDestroy: %s", msg);
    return PM_OK;
}

// The group as RCCL itself reports it (not the numbers the caller passed to pm_comm_init).
extern "C" int pm_comm_info(const pm_comm* c, int32_t* nranks, int32_t* rank, int32_t* device) {
    PM_REQUIRE(c && c->comm, PM_E_ARG, "pm_comm_info: null communicator");
    PM_REQUIRE(c->rccl.comm_count && c->rccl.comm_user_rank && c->rccl.comm_device, PM_E_COMM,
               "pm_comm_info: RCCL lacks ncclCommCount / ncclCommUserRank / ncclCommCuDevice");
    int n = 0, r = 0, d = 0;
    ncclResult_t e = c->rccl.comm_count(c->comm, &n);
    if (!e) e = c->rccl.comm_user_rank(c->comm, &r);
    if (!e) e = c->rccl.comm_device(c->comm, &d);
    PM_REQUIRE(e == 0, PM_E_COMM, "ncclCommCount / UserRank / CuDevice: %s", c->rccl.error_string(e));
    if (nranks) *nranks = n;
    if (rank) *rank = r;
    if (device) *device = d;
    return PM_OK;
}

extern "C" int pm_comm_allreduce_f32(pm_comm* c, float* buf, int64_t n, void* stream) {
    PM_REQUIRE(c && c->comm && buf && n >= 0, PM_E_ARG, "pm_comm_allreduce_f32: null comm / buffer");
    if (n == 0) return PM_OK;
    const ncclResult_t e = c->rccl.all_reduce(buf, buf, (size_t)n, kNcclFloat32, kNcclSum, c->comm, pm_stream(stream));
    PM_REQUIRE(e == 0, PM_E_COMM, "ncclAllReduce(%lld floats): %s", (long long)n, c->rccl.error_string(e));
    return PM_OK;
}

// The sharded DQN vector step (the Python sequence of SelfPlayLearner.step / _step_multi for
// world > 1, overlapped): actenv, then per update u: [resample] + learn_ex (u = 0: with the next
// step's side-A act) + all-reduce of sp->grad + apply_ex; U > 1 closes with commit.
extern "C" int pm_selfplay_step_sharded(const pm_selfplay* sp, pm_comm* c, int32_t updates, void* stream) {
    PM_REQUIRE(sp && c, PM_E_ARG, "pm_selfplay_step_sharded: null learner / comm");
    PM_REQUIRE(updates >= 1, PM_E_ARG, "pm_selfplay_step_sharded: updates=%d", updates);
    PM_REQUIRE(!sp->fuse_apply, PM_E_ARG, "pm_selfplay_step_sharded: the learner fuses its apply (world 1)");
    PM_REQUIRE(sp->world == c->nranks, PM_E_ARG, "pm_selfplay_step_sharded: learner world %d vs communicator %d",
               sp->world, c->nranks);
    const int32_t n_grad = PM_GRAD_LEN;  // sp->grad: head gradients, finished episodes, updated flag, pad
    int rc = pm_selfplay_actenv(sp, stream);
    for (int u = 0; !rc && u < updates; ++u) {
        const int32_t mode = updates == 1 ? (PM_UPD_FIRST | PM_UPD_LAST) : (u == 0 ? PM_UPD_FIRST : 0);
        if (u) rc = pm_selfplay_resample(sp, stream);
        if (!rc) rc = pm_selfplay_learn_ex(sp, mode, u == 0, stream);
        if (!rc) rc = pm_comm_allreduce_f32(c, sp->grad, n_grad, stream);
        if (!rc) rc = pm_selfplay_apply_ex(sp, mode, stream);
    }
    if (!rc && updates > 1) rc = pm_selfplay_commit(sp, stream);
    return rc;
}

// The sharded QNetRNN vector step (RNNSelfPlayLearner.step for world > 1): rollout, then per update
// u: [sample(u)] + grads + all-reduce of d->grad (gradients + contributing-rank count) + apply.
extern "C" int pm_rnn_selfplay_step_sharded(const pm_rnn_selfplay* sp, const pm_drqn* d, pm_comm* c,
                                            int32_t updates, void* stream) {
    PM_REQUIRE(sp && d && c, PM_E_ARG, "pm_rnn_selfplay_step_sharded: null learner / drqn / comm");
    PM_REQUIRE(updates >= 1, PM_E_ARG, "pm_rnn_selfplay_step_sharded: updates=%d", updates);
    int rc = pm_rnn_selfplay_rollout(sp, d, stream);
    for (int u = 0; !rc && u < updates; ++u) {
        if (u) rc = pm_rnn_selfplay_sample(sp, d, u, stream);
        if (!rc) rc = pm_drqn_grads(d, stream);
        if (!rc) rc = pm_comm_allreduce_f32(c, d->grad, PM_RNN_NPARAM + 4, stream);
        if (!rc) rc = pm_drqn_apply(d, stream);
    }
    return rc;
}
