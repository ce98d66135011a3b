// psim_comm.h -- the collective layer of a multi-rank handle (shard_world >
// 1, one shard per rank).  Every cross-rank step of the
// engine goes through this interface:
//   all_to_all_u64  the per-owner record counts of a round (exchange_rccl)
//   exchange        the records themselves, grouped point-to-point sends and
//                   receives of byte ranges (exchange_rccl)
//   all_reduce      the round's stats (sum), the overlay statistics (sum, max)
//   all_gather      the stop lists of leave/1, the active rows of the overlay
//                   statistics
// Two implementations:
//   RcclComm      the product backend: RCCL over xGMI, one process per GPU,
//                 every call enqueued on the caller's stream;
//   LoopbackComm  TEST VEHICLE: the ranks are threads of one process driving
//                 handles on one device; a call synchronises the caller's
//                 stream, meets the other ranks at a host barrier and moves
//                 the data with device copies.  It exists so that the rank
//                 code path -- the owner partition's offsets, the count
//                 all-to-all and its one host read, the self-copy, the
//                 receive grouping, the stats reduce, the stop-list gather --
//                 runs on a one-GPU box (RCCL refuses two ranks on one
//                 device); bench.py never selects it.
// Host code only.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/partisan_gpu_sim.h"

namespace psim {

#define TRYC(x)                  \
    do {                         \
        int rc_ = (x);           \
        if (rc_) return rc_;     \
    } while (0)

struct Xfer {
    int peer;
    void* ptr;        // device memory
    size_t bytes;
};

enum class CType { U8, U32, U64 };
enum class COp { SUM, MAX };

struct Comm {
    int rank = 0, world = 1;
    virtual ~Comm() {}
    // recv[g * count + i] = rank g's send[rank * count + i]
    virtual int all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t count, hipStream_t st) = 0;
    // grouped point-to-point: each send to peer g matches g's receive from
    // this rank, byte for byte (zero-byte entries are left out by the caller)
    virtual int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) = 0;
    // in place
    virtual int all_reduce(void* buf, size_t count, CType t, COp op, hipStream_t st) = 0;
    // recv[g * bytes ..] = rank g's send (send may be recv + rank * bytes)
    virtual int all_gather(const void* send, void* recv, size_t bytes, hipStream_t st) = 0;
};

// ------------------------------------------------------------------ RCCL --
struct RcclComm : Comm {
    ncclComm_t c = nullptr;
    ~RcclComm() override {
        if (c) ncclCommDestroy(c);
    }
    static int check(ncclResult_t r, const char* what) {
        if (r == ncclSuccess) return PSIM_OK;
        std::fprintf(stderr, "psim: %s failed: %s\n", what, ncclGetErrorString(r));
        return PSIM_ECOMM;
    }
    int init(const void* id_bytes, int rank_, int world_) {
        rank = rank_; world = world_;
        ncclUniqueId id;
        memcpy(&id, id_bytes, sizeof id);
        const ncclResult_t r = ncclCommInitRank(&c, world, id, rank);
        if (r != ncclSuccess) c = nullptr;
        return check(r, "ncclCommInitRank");
    }
    int all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t count, hipStream_t st) override {
        return check(ncclAllToAll(send, recv, count, ncclUint64, c, st), "ncclAllToAll");
    }
    int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) override {
        int rc = check(ncclGroupStart(), "ncclGroupStart");
        // (sends and receives interleaved by peer inside one group)
        for (const Xfer& x : sends)
            if (!rc) rc = check(ncclSend(x.ptr, x.bytes, ncclUint8, x.peer, c, st), "ncclSend");
        for (const Xfer& x : recvs)
            if (!rc) rc = check(ncclRecv(x.ptr, x.bytes, ncclUint8, x.peer, c, st), "ncclRecv");
        const int rc2 = check(ncclGroupEnd(), "ncclGroupEnd");
        return rc ? rc : rc2;
    }
    static ncclDataType_t dt(CType t) { return t == CType::U8 ? ncclUint8 : t == CType::U32 ? ncclUint32 : ncclUint64; }
    int all_reduce(void* buf, size_t count, CType t, COp op, hipStream_t st) override {
        return check(ncclAllReduce(buf, buf, count, dt(t), op == COp::SUM ? ncclSum : ncclMax, c, st), "ncclAllReduce");
    }
    int all_gather(const void* send, void* recv, size_t bytes, hipStream_t st) override {
        return check(ncclAllGather(send, recv, bytes, ncclUint8, c, st), "ncclAllGather");
    }
};

// -------------------------------------------------------------- loopback --
// The ranks of one loopback world meet at a host barrier; each posts its
// arguments, reads the others' after the first barrier, and a second barrier
// keeps every buffer alive until all ranks are done with it.
struct LoopWorld {
    int world = 0;
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;
    int arrived = 0;
    struct Post {
        const void* send = nullptr;
        void* recv = nullptr;
        std::vector<Xfer> sends;
    };
    std::vector<Post> posts;
    bool broken = false;
    // every rank of the world arrives, or (a rank that failed before the
    // collective never comes) after 120 s the world is broken and every
    // later call fails at once instead of hanging its thread
    int barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return PSIM_ECOMM;
        const uint64_t g = gen;
        if (++arrived == world) {
            arrived = 0;
            gen++;
            cv.notify_all();
            return PSIM_OK;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            std::fprintf(stderr, "psim: loopback: a rank never reached the collective\n");
            return PSIM_ECOMM;
        }
        return PSIM_OK;
    }
};

// loopback id bytes: this magic, then the world's key (psim_loopback_comm_id)
constexpr char kLoopMagic[16] = "PSIM-LOOPBACK-1";

struct LoopRegistry {
    std::mutex mu;
    uint64_t next = 1;
    std::map<uint64_t, std::weak_ptr<LoopWorld>> worlds;
    static LoopRegistry& get() {
        static LoopRegistry r;
        return r;
    }
};

struct LoopbackComm : Comm {
    std::shared_ptr<LoopWorld> w;
    static bool is_loopback_id(const void* id) { return id && memcmp(id, kLoopMagic, sizeof kLoopMagic) == 0; }
    int init(const void* id_bytes, int rank_, int world_) {
        rank = rank_; world = world_;
        uint64_t key;
        memcpy(&key, (const char*)id_bytes + sizeof kLoopMagic, sizeof key);
        LoopRegistry& reg = LoopRegistry::get();
        std::lock_guard<std::mutex> lk(reg.mu);
        auto it = reg.worlds.find(key);
        if (it == reg.worlds.end()) return PSIM_EINVAL;          // (not an id of this process)
        w = it->second.lock();
        if (!w) {
            w = std::make_shared<LoopWorld>();
            w->world = world;
            w->posts.resize(world);
            it->second = w;
        }
        return w->world == world ? PSIM_OK : PSIM_EINVAL;
    }
    static int sync(hipStream_t st) {
        const hipError_t e = hipStreamSynchronize(st);
        if (e == hipSuccess) return PSIM_OK;
        std::fprintf(stderr, "psim: loopback: %s\n", hipGetErrorString(e));
        return PSIM_EDEVICE;
    }
    static int copy(void* dst, const void* src, size_t bytes, hipStream_t st) {
        if (!bytes || dst == src) return PSIM_OK;
        const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) return PSIM_OK;
        std::fprintf(stderr, "psim: loopback copy: %s\n", hipGetErrorString(e));
        return PSIM_EDEVICE;
    }
    // the collective's frame: this rank's inputs are ready, everyone has
    // posted; body(); every copy done; everyone is past its reads.  A failing
    // body still meets the second barrier (no rank is left waiting).
    template <class F>
    int frame(hipStream_t st, const LoopWorld::Post& p, F body) {
        int rc = sync(st);
        w->posts[rank] = p;
        TRYC(w->barrier());
        if (!rc) rc = body();
        if (!rc) rc = sync(st);
        const int rb = w->barrier();
        return rc ? rc : rb;
    }
    int all_to_all_u64(const uint64_t* send, uint64_t* recv, size_t count, hipStream_t st) override {
        LoopWorld::Post p;
        p.send = send;
        return frame(st, p, [&] {
            for (int g = 0; g < world; g++)
                TRYC(copy(recv + (size_t)g * count, (const uint64_t*)w->posts[g].send + (size_t)rank * count,
                          count * 8, st));
            return PSIM_OK;
        });
    }
    int exchange(const std::vector<Xfer>& sends, const std::vector<Xfer>& recvs, hipStream_t st) override {
        LoopWorld::Post p;
        p.sends = sends;
        return frame(st, p, [&] {
            // the k-th receive from a peer takes the peer's k-th send to this
            // rank (point-to-point order, as RCCL matches a group's messages)
            std::map<int, int> nth;
            for (const Xfer& r : recvs) {
                const Xfer* m = nullptr;
                int k = nth[r.peer]++;
                for (const Xfer& s : w->posts[r.peer].sends)
                    if (s.peer == rank && k-- == 0) { m = &s; break; }
                if (!m || m->bytes != r.bytes) {
                    std::fprintf(stderr, "psim: loopback: rank %d expects %zu B from %d, which sends %zu\n", rank,
                                 r.bytes, r.peer, m ? m->bytes : (size_t)0);
                    return PSIM_ECOMM;
                }
                TRYC(copy(r.ptr, m->ptr, r.bytes, st));
            }
            return PSIM_OK;
        });
    }
    int all_reduce(void* buf, size_t count, CType t, COp op, hipStream_t st) override {
        const size_t sz = t == CType::U8 ? 1 : t == CType::U32 ? 4 : 8;
        std::vector<uint8_t> all((size_t)world * count * sz);
        LoopWorld::Post p;
        p.recv = buf;
        // read every rank's buffer between the barriers, reduce, then write
        // this rank's after the second barrier (no one reads it any more)
        int rc = frame(st, p, [&] {
            for (int g = 0; g < world; g++) {
                const hipError_t e = hipMemcpyAsync(all.data() + (size_t)g * count * sz, w->posts[g].recv,
                                                    count * sz, hipMemcpyDeviceToHost, st);
                if (e != hipSuccess) return PSIM_EDEVICE;
            }
            return PSIM_OK;
        });
        if (rc) return rc;
        std::vector<uint8_t> out(count * sz);
        for (size_t i = 0; i < count; i++) {
            uint64_t acc = 0;
            for (int g = 0; g < world; g++) {
                uint64_t v = 0;
                memcpy(&v, all.data() + ((size_t)g * count + i) * sz, sz);
                acc = g == 0 ? v : op == COp::SUM ? acc + v : (v > acc ? v : acc);
            }
            memcpy(out.data() + i * sz, &acc, sz);
        }
        if (hipMemcpyAsync(buf, out.data(), count * sz, hipMemcpyHostToDevice, st) != hipSuccess) return PSIM_EDEVICE;
        return sync(st);
    }
    int all_gather(const void* send, void* recv, size_t bytes, hipStream_t st) override {
        LoopWorld::Post p;
        p.send = send;
        return frame(st, p, [&] {
            for (int g = 0; g < world; g++)
                TRYC(copy((uint8_t*)recv + (size_t)g * bytes, w->posts[g].send, bytes, st));
            return PSIM_OK;
        });
    }
};

// psim_loopback_comm_id: a new loopback world's id bytes
inline int loopback_new_id(void* buf, size_t cap) {
    if (!buf || cap < sizeof(ncclUniqueId) || sizeof(ncclUniqueId) < sizeof kLoopMagic + 8) return PSIM_EINVAL;
    LoopRegistry& reg = LoopRegistry::get();
    std::lock_guard<std::mutex> lk(reg.mu);
    const uint64_t key = reg.next++;
    reg.worlds[key];                                   // (created by the first rank that attaches)
    memset(buf, 0, sizeof(ncclUniqueId));
    memcpy(buf, kLoopMagic, sizeof kLoopMagic);
    memcpy((char*)buf + sizeof kLoopMagic, &key, sizeof key);
    return PSIM_OK;
}

}  // namespace psim
