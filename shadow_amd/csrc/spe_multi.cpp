// spe_multi.cpp -- multi-device path tables in one process.
//
// Shadow runs as ONE process (shd-master.c:390-394: "For now we only have one
// slave"), so the drop-in cannot rely on one rank per GPU: the library itself
// drives every device of the node.  A multi-device table is one part table per
// device, each over a contiguous share of the 64-source blocks (the sources are
// independent rows: no exchange during the build), built concurrently from one
// host thread per device on that device's own stream.  The parts write their
// {latency, reliability} records straight into a full-size replica on their own
// device (at their share's offset), and one all-gather then fills every replica:
//   RCCL  ncclCommInitAll over the device list; per gather round one group of
//         ncclSend / ncclRecv pairs, every share's chunk from its owner to every
//         other device in place -- N - 1 concurrent point-to-point transfers into
//         each device, one per xGMI link (SPE_RCCL_BCAST=1: one ncclBroadcast
//         per root instead, RCCL's ring / tree);
//   PEER  hipMemcpyPeerAsync of every share to every other device, each source
//         device on its own stream so a receiver's N - 1 copies run concurrently
//         (also the path for a device list that repeats a GPU, which RCCL refuses).
// Next hop and hop count stay with the device that built them.  RCCL is loaded
// with dlopen on first use, so single-device users never load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "spe_internal.h"

namespace spe {

namespace {

constexpr int32_t kWave = 64;

struct Rccl {
    bool tried = false;
    bool ok = false;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl& rccl_lib() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    // the process's RCCL if one is loaded already (e.g. by PyTorch), else ROCm's
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW);
    if (!h) return r;
    r.comm_init_all = (decltype(r.comm_init_all))dlsym(h, "ncclCommInitAll");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.broadcast = (decltype(r.broadcast))dlsym(h, "ncclBroadcast");
    r.send = (decltype(r.send))dlsym(h, "ncclSend");   // optional: broadcasts without them
    r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.ok = r.comm_init_all && r.comm_destroy && r.all_gather && r.broadcast && r.group_start && r.group_end &&
           r.error_string;
    return r;
}

int hip_fail(const char* what, hipError_t e) { return set_error(SPE_EHIP, std::string(what) + ": " + hipGetErrorString(e)); }

}  // namespace

struct MultiDev {
    int32_t A = 0, nblk = 0, n = 0;
    int32_t cb = 0;                        // blocks per share of the sharded region
    int32_t S = 0;                         // sharded blocks [0, S); every device builds [S, nblk) itself
    int32_t span = 0;                      // replica blocks: max(n * cb, nblk) (pure sharding pads the last share)
    int32_t chunk = 1;                     // blocks a share sends per gather round (one build launch)
    int32_t gather = SPE_GATHER_PEER;
    double shared_fraction = 1.0;
    std::vector<int32_t> devs;
    std::vector<int32_t> b0, b1;           // share of each device (clipped to S)
    spe_graph* home = nullptr;             // the caller's graph (not owned)
    std::vector<spe_graph*> graphs;        // per device: home, or a clone on that device
    std::vector<spe_table*> parts;         // the share's part table; nullptr for an empty share
    std::vector<spe_table*> lparts;        // the local remainder's part table (nullptr: S == nblk)
    std::vector<void*> replica;            // full {lat, rel} span per device
    std::vector<void*> next, hops;         // the device's own share
    std::vector<void*> lnext, lhops;       // the device's own copy of the local remainder
    std::vector<hipStream_t> streams;      // per device: the gather stream
    std::vector<std::vector<hipStream_t>> pstreams;   // PEER: [receiver][source device] copy streams
    std::vector<std::vector<hipEvent_t>> pevents;     // ... and their completion events (joined into streams)
    std::vector<ncclComm_t> comms;
    bool built = false;
    bool fw = false;                       // FW-engine parts: one closure across the devices
    spe_build_stats stats{};

    size_t blk_elems() const { return (size_t)A * kWave; }
    size_t blk_bytes() const { return blk_elems() * 2 * sizeof(double); }
};

// The a-priori one-device build time the split model uses when the caller gives
// none: relaxation ~1.5e-10 s per (source, relaxation vertex) and rows at ~3.4 TB/s
// of 22-B entries (within ~25 % of the measured C3 / C4 tables).
static double build_time_estimate(int32_t n_relax, int32_t A) {
    return 1.5e-10 * (double)n_relax * (double)A + 22.0 * (double)A * (double)A / 3.4e12;
}

double multi_shared_fraction(int32_t n_dev, double t1_s, double span_bytes, double gather_bps) {
    if (n_dev <= 1 || t1_s <= 0.0 || gather_bps <= 0.0) return 1.0;
    const double x = t1_s * n_dev / ((n_dev - 1) * (span_bytes / gather_bps + t1_s));
    return std::min(1.0, std::max(0.0, x));
}

int multi_create(spe_graph* g, const int32_t* attached, int32_t A, const spe_table_opts& o, MultiDev** out) {
    *out = nullptr;
    if (o.block_begin || o.block_end || o.ext_latrel || o.ext_next_hop || o.ext_hops || o.owner_rank || o.want_aux)
        return set_error(SPE_EUNSUPPORTED, "a multi-device table owns every block and its own storage "
                                           "(no block range, external storage, owner replay or want_aux)");
    if (o.gather < SPE_GATHER_AUTO || o.gather > SPE_GATHER_PEER) return set_error(SPE_EINVAL, "unknown gather mode");
    if (o.shared_fraction < 0.0 || o.shared_fraction > 1.0) return set_error(SPE_EINVAL, "shared_fraction must be in [0, 1]");
    spe_graph_info gi = SPE_STRUCT_INIT(spe_graph_info);
    spe_graph_info_get(g, &gi);
    auto* m = new MultiDev();
    m->home = g;
    m->A = A;
    m->n = o.n_devices;
    m->devs.assign(o.devices, o.devices + o.n_devices);
    m->nblk = (A + kWave - 1) / kWave;
    // the split: FW parts share one closure over the shares, so they never split
    double x = 1.0;
    if (o.engine != SPE_ENGINE_FW) {
        if (o.shared_fraction > 0.0) {
            x = o.shared_fraction;
        } else {
            const double t1 = o.build_seconds_hint > 0.0 ? o.build_seconds_hint : build_time_estimate(gi.n_relax_vertices, A);
            const double bps = (o.gather_gbps > 0.0 ? o.gather_gbps : 300.0) * 1e9;
            x = multi_shared_fraction(m->n, t1, (double)m->nblk * m->blk_bytes(), bps);
        }
    }
    m->shared_fraction = x;
    m->b0.resize(m->n);
    m->b1.resize(m->n);
    spe_device_split(A, m->n, x, m->b0.data(), m->b1.data(), &m->S);
    m->cb = m->n > 0 ? std::max(0, m->b1[0] - m->b0[0]) : 0;
    if (x >= 1.0) m->cb = (m->nblk + m->n - 1) / m->n;   // shares padded to equal size (the last one short)
    m->span = std::max(m->n * m->cb, m->nblk);
    bool distinct = true;
    for (int i = 0; i < m->n; ++i)
        for (int j = 0; j < i; ++j) distinct &= m->devs[i] != m->devs[j];
    if (o.gather == SPE_GATHER_RCCL && !distinct) {
        delete m;
        return set_error(SPE_EUNSUPPORTED, "RCCL needs distinct devices (a repeated device: use SPE_GATHER_PEER)");
    }
    m->gather = o.gather == SPE_GATHER_PEER || !distinct ? SPE_GATHER_PEER
                : (rccl_lib().ok ? SPE_GATHER_RCCL : (o.gather == SPE_GATHER_RCCL ? -1 : SPE_GATHER_PEER));
    if (m->gather < 0) {
        delete m;
        return set_error(SPE_EUNSUPPORTED, "librccl.so.1 could not be loaded");
    }
    const int32_t nd = m->n;
    m->graphs.assign(nd, nullptr);
    m->parts.assign(nd, nullptr);
    m->lparts.assign(nd, nullptr);
    m->replica.assign(nd, nullptr);
    m->next.assign(nd, nullptr);
    m->hops.assign(nd, nullptr);
    m->lnext.assign(nd, nullptr);
    m->lhops.assign(nd, nullptr);
    m->streams.assign(nd, nullptr);
    int r = SPE_OK;
    const size_t rep_bytes = (size_t)m->span * m->blk_bytes();
    const size_t own = (size_t)m->cb * m->blk_elems();
    const size_t loc = (size_t)(m->nblk - std::min(m->nblk, m->S)) * m->blk_elems();
    for (int d = 0; d < nd && !r; ++d) {
        if (m->devs[d] == gi.device) {
            m->graphs[d] = g;
        } else if ((r = graph_clone(g, m->devs[d], &m->graphs[d]))) {
            break;
        }
        hipError_t e = hipSetDevice(m->devs[d]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->streams[d], hipStreamNonBlocking);
        if (m->gather == SPE_GATHER_PEER) {
            m->pstreams.resize(nd);
            m->pevents.resize(nd);
            m->pstreams[d].assign(nd, nullptr);
            m->pevents[d].assign(nd, nullptr);
            for (int q = 0; q < nd && e == hipSuccess; ++q) {
                if (q == d) continue;
                e = hipStreamCreateWithFlags(&m->pstreams[d][q], hipStreamNonBlocking);
                if (e == hipSuccess) e = hipEventCreateWithFlags(&m->pevents[d][q], hipEventDisableTiming);
            }
        }
        if (e == hipSuccess) e = hipMalloc(&m->replica[d], rep_bytes);
        if (e == hipSuccess) e = hipMalloc(&m->next[d], std::max<size_t>(1, own) * sizeof(int32_t));
        if (e == hipSuccess) e = hipMalloc(&m->hops[d], std::max<size_t>(1, own) * sizeof(uint16_t));
        if (e == hipSuccess && loc) e = hipMalloc(&m->lnext[d], loc * sizeof(int32_t));
        if (e == hipSuccess && loc) e = hipMalloc(&m->lhops[d], loc * sizeof(uint16_t));
        if (e != hipSuccess) {
            r = hip_fail("multi-device table storage", e);
            break;
        }
        spe_table_opts po = o;
        po.devices = nullptr;
        po.n_devices = 0;
        po.ext_filled = 0;
        if (m->b1[d] > m->b0[d]) {
            po.block_begin = m->b0[d];
            po.block_end = m->b1[d];
            po.ext_latrel = (char*)m->replica[d] + (size_t)m->b0[d] * m->blk_bytes();
            po.ext_next_hop = m->next[d];
            po.ext_hops = m->hops[d];
            r = spe_table_create(m->graphs[d], attached, A, &po, &m->parts[d]);
            if (!r) {
                spe_table_layout pl = SPE_STRUCT_INIT(spe_table_layout);
                spe_table_layout_get(m->parts[d], &pl);
                FwPart fp;
                m->fw = pl.engine == SPE_ENGINE_FW && fw_part(m->parts[d], &fp) == SPE_OK;   // not for DIRECT tables
                m->chunk = std::max(1, pl.groups_per_launch);
            }
        }
        if (!r && loc) {   // the local remainder, built in place on this device
            po.block_begin = m->S;
            po.block_end = m->nblk;
            po.ext_latrel = (char*)m->replica[d] + (size_t)m->S * m->blk_bytes();
            po.ext_next_hop = m->lnext[d];
            po.ext_hops = m->lhops[d];
            r = spe_table_create(m->graphs[d], attached, A, &po, &m->lparts[d]);
        }
    }
    if (!r && m->gather == SPE_GATHER_RCCL) {
        m->comms.assign(nd, nullptr);
        const ncclResult_t nr = rccl_lib().comm_init_all(m->comms.data(), nd, m->devs.data());
        if (nr != ncclSuccess) {
            m->comms.clear();
            r = set_error(SPE_EHIP, std::string("ncclCommInitAll: ") + rccl_lib().error_string(nr));
        }
    }
    if (r) {
        multi_free(m);
        return r;
    }
    *out = m;
    return SPE_OK;
}

void multi_free(MultiDev* m) {
    if (!m) return;
    for (ncclComm_t c : m->comms)
        if (c) rccl_lib().comm_destroy(c);
    for (int d = 0; d < m->n; ++d) {
        if (m->parts[d]) spe_table_free(m->parts[d]);
        if (m->lparts[d]) spe_table_free(m->lparts[d]);
        (void)hipSetDevice(m->devs[d]);
        if (m->streams[d]) (void)hipStreamSynchronize(m->streams[d]);
        for (void* p : {m->replica[d], m->next[d], m->hops[d], m->lnext[d], m->lhops[d]})
            if (p) (void)hipFree(p);
        if (m->streams[d]) (void)hipStreamDestroy(m->streams[d]);
        if (d < (int)m->pstreams.size())
            for (int q = 0; q < (int)m->pstreams[d].size(); ++q) {
                if (m->pstreams[d][q]) {
                    (void)hipStreamSynchronize(m->pstreams[d][q]);
                    (void)hipStreamDestroy(m->pstreams[d][q]);
                }
                if (m->pevents[d][q]) (void)hipEventDestroy(m->pevents[d][q]);
            }
        if (m->graphs[d] && m->graphs[d] != m->home) spe_graph_free(m->graphs[d]);
    }
    delete m;
}

// Round k of the gather: every share's chunk k -- blocks [b0 + k c, b0 + (k + 1) c)
// clipped to the share -- to every other device, in place on every replica (the
// chunks of a round are not contiguous, so an all-gather does not fit).  RCCL: one
// group of send / receive pairs (each device receives its N - 1 chunks over N - 1
// links at once), or one ncclBroadcast per root; PEER: each device pulls the other
// chunks, one stream per source device, joined into its gather stream.  The chunks
// were built synchronously before.
static int gather_round(MultiDev* m, int32_t k) {
    static const bool bcast = [] {
        const char* e = getenv("SPE_RCCL_BCAST");
        return e && *e && *e != '0';
    }();
    if (m->gather == SPE_GATHER_RCCL && !bcast && rccl_lib().send && rccl_lib().recv) {
        Rccl& R = rccl_lib();
        R.group_start();
        ncclResult_t nr = ncclSuccess;
        for (int root = 0; root < m->n && nr == ncclSuccess; ++root) {
            const int32_t c0 = std::min(m->b1[root], m->b0[root] + k * m->chunk);
            const int32_t c1 = std::min(m->b1[root], c0 + m->chunk);
            if (c1 <= c0) continue;
            const size_t off = (size_t)c0 * m->blk_bytes();
            const size_t cnt = (size_t)(c1 - c0) * m->blk_elems() * 2;
            for (int d = 0; d < m->n && nr == ncclSuccess; ++d) {
                if (d == root) continue;
                if (hipSetDevice(m->devs[root]) != hipSuccess) {
                    R.group_end();
                    return set_error(SPE_EHIP, "hipSetDevice");
                }
                nr = R.send((char*)m->replica[root] + off, cnt, ncclDouble, d, m->comms[root], m->streams[root]);
                if (nr != ncclSuccess) break;
                if (hipSetDevice(m->devs[d]) != hipSuccess) {
                    R.group_end();
                    return set_error(SPE_EHIP, "hipSetDevice");
                }
                nr = R.recv((char*)m->replica[d] + off, cnt, ncclDouble, root, m->comms[d], m->streams[d]);
            }
        }
        const ncclResult_t ne = R.group_end();
        if (nr != ncclSuccess || ne != ncclSuccess)
            return set_error(SPE_EHIP, std::string("ncclSend/ncclRecv: ") + R.error_string(nr != ncclSuccess ? nr : ne));
        return SPE_OK;
    }
    if (m->gather == SPE_GATHER_RCCL) {
        Rccl& R = rccl_lib();
        R.group_start();
        ncclResult_t nr = ncclSuccess;
        for (int root = 0; root < m->n && nr == ncclSuccess; ++root) {
            const int32_t c0 = std::min(m->b1[root], m->b0[root] + k * m->chunk);
            const int32_t c1 = std::min(m->b1[root], c0 + m->chunk);
            if (c1 <= c0) continue;
            const size_t off = (size_t)c0 * m->blk_bytes();
            const size_t cnt = (size_t)(c1 - c0) * m->blk_elems() * 2;
            for (int d = 0; d < m->n && nr == ncclSuccess; ++d) {
                if (hipSetDevice(m->devs[d]) != hipSuccess) {
                    R.group_end();
                    return set_error(SPE_EHIP, "hipSetDevice");
                }
                char* buf = (char*)m->replica[d] + off;
                nr = R.broadcast(buf, buf, cnt, ncclDouble, root, m->comms[d], m->streams[d]);
            }
        }
        const ncclResult_t ne = R.group_end();
        if (nr != ncclSuccess || ne != ncclSuccess)
            return set_error(SPE_EHIP, std::string("ncclBroadcast: ") + R.error_string(nr != ncclSuccess ? nr : ne));
        return SPE_OK;
    }
    for (int e = 0; e < m->n; ++e) {   // device e pulls every other share's chunk
        if (hipSetDevice(m->devs[e]) != hipSuccess) return set_error(SPE_EHIP, "hipSetDevice");
        for (int d = 0; d < m->n; ++d) {
            if (d == e) continue;
            const int32_t c0 = std::min(m->b1[d], m->b0[d] + k * m->chunk);
            const int32_t c1 = std::min(m->b1[d], c0 + m->chunk);
            if (c1 <= c0) continue;
            const size_t off = (size_t)c0 * m->blk_bytes();
            hipError_t he = hipMemcpyPeerAsync((char*)m->replica[e] + off, m->devs[e],
                                               (const char*)m->replica[d] + off, m->devs[d],
                                               (size_t)(c1 - c0) * m->blk_bytes(), m->pstreams[e][d]);
            if (he == hipSuccess) he = hipEventRecord(m->pevents[e][d], m->pstreams[e][d]);
            if (he == hipSuccess) he = hipStreamWaitEvent(m->streams[e], m->pevents[e][d], 0);
            if (he != hipSuccess) return hip_fail("hipMemcpyPeerAsync", he);
        }
    }
    return SPE_OK;
}

// ---- FW engine parts: the closure is computed ONCE across the devices instead
// of once per part (SURVEY §8e "dense FW: one exchange step per pivot block").
// The closure's ld / 64 row blocks are dealt contiguously to the devices; per
// pivot block kb the owner of row block kb relaxes the diagonal tile and the
// pivot row panel, the panel's (D, R) rows are broadcast to every device (RCCL
// ncclBroadcast over xGMI, in place; or peer copies), and each device relaxes
// its own rows' column panel and remaining tiles.  Finally every device
// broadcasts its rows' (D, N) so that each holds the whole closure for its
// part's row walks (R is not needed there: the rows re-fold in path order).
namespace {
struct FwBcast {
    const MultiDev* m;
    std::vector<FwPart>& P;
    std::vector<hipEvent_t>& ev;      // per device: its copies issued / its rows ready to read
    std::vector<hipEvent_t>& ready;   // per device: every kernel it queued so far (destination side)
    bool rccl;
    // rows [r0, r1) of the arrays in `which` (bit 0 D, 1 R, 2 N) from device `root` to every other
    int rows(int root, int64_t r0, int64_t r1, int which) {
        const int64_t ld = P[root].ld;
        const size_t off = (size_t)r0 * (size_t)ld, cnt = (size_t)(r1 - r0) * (size_t)ld;
        if (cnt == 0) return SPE_OK;
        if (rccl) {
            Rccl& R = rccl_lib();
            R.group_start();
            ncclResult_t nr = ncclSuccess;
            for (int d = 0; d < m->n && nr == ncclSuccess; ++d) {
                if (hipSetDevice(P[d].device) != hipSuccess) return set_error(SPE_EHIP, "hipSetDevice");
                hipStream_t s = (hipStream_t)P[d].stream;
                if (which & 1) nr = R.broadcast(P[d].D + off, P[d].D + off, cnt, ncclDouble, root, m->comms[d], s);
                if (nr == ncclSuccess && (which & 2))
                    nr = R.broadcast(P[d].R + off, P[d].R + off, cnt, ncclDouble, root, m->comms[d], s);
                if (nr == ncclSuccess && (which & 4))
                    nr = R.broadcast(P[d].N + off, P[d].N + off, cnt, ncclInt32, root, m->comms[d], s);
            }
            const ncclResult_t ne = R.group_end();
            if (nr != ncclSuccess || ne != ncclSuccess)
                return set_error(SPE_EHIP, std::string("ncclBroadcast: ") + R.error_string(nr != ncclSuccess ? nr : ne));
            return SPE_OK;
        }
        // peer copies on the root's stream (its later kernels overwrite these rows),
        // ordered after everything each destination queued before (a destination's
        // earlier kernels -- its init, or the column panel / rest of the previous
        // pivot -- still read or write the rows the copy lands in), then every
        // other device's stream waits for the copies
        const FwPart& o = P[root];
        for (int d = 0; d < m->n; ++d) {
            if (d == root) continue;
            if (hipSetDevice(P[d].device) != hipSuccess) return set_error(SPE_EHIP, "hipSetDevice");
            const hipError_t e = hipEventRecord(ready[d], (hipStream_t)P[d].stream);
            if (e != hipSuccess) return hip_fail("hipEventRecord (FW destination)", e);
        }
        if (hipSetDevice(o.device) != hipSuccess) return set_error(SPE_EHIP, "hipSetDevice");
        hipStream_t so = (hipStream_t)o.stream;
        for (int d = 0; d < m->n; ++d) {
            if (d == root) continue;
            const hipError_t e = hipStreamWaitEvent(so, ready[d], 0);
            if (e != hipSuccess) return hip_fail("hipStreamWaitEvent (FW destination)", e);
        }
        for (int d = 0; d < m->n; ++d) {
            if (d == root) continue;
            hipError_t e = hipSuccess;
            if (which & 1) e = hipMemcpyPeerAsync(P[d].D + off, P[d].device, o.D + off, o.device, cnt * 8, so);
            if (e == hipSuccess && (which & 2))
                e = hipMemcpyPeerAsync(P[d].R + off, P[d].device, o.R + off, o.device, cnt * 8, so);
            if (e == hipSuccess && (which & 4))
                e = hipMemcpyPeerAsync(P[d].N + off, P[d].device, o.N + off, o.device, cnt * 4, so);
            if (e != hipSuccess) return hip_fail("hipMemcpyPeerAsync (FW rows)", e);
        }
        hipError_t e = hipEventRecord(ev[root], so);
        if (e != hipSuccess) return hip_fail("hipEventRecord", e);
        for (int d = 0; d < m->n; ++d) {
            if (d == root) continue;
            if (hipSetDevice(P[d].device) != hipSuccess) return set_error(SPE_EHIP, "hipSetDevice");
            e = hipStreamWaitEvent((hipStream_t)P[d].stream, ev[root], 0);
            if (e != hipSuccess) return hip_fail("hipStreamWaitEvent", e);
        }
        return SPE_OK;
    }
};
}  // namespace

static int fw_closure_multi(MultiDev* m, double* seconds) {
    std::vector<FwPart> P(m->n);
    for (int d = 0; d < m->n; ++d) {
        // an empty share (more devices than source blocks): every part computes its own closure
        if (!m->parts[d]) return SPE_OK;
        if (int r = fw_part(m->parts[d], &P[d])) return r;
    }
    bool done = true;
    for (auto& p : P) done &= *p.done;
    if (done) return SPE_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const int32_t nb = (int32_t)(P[0].ld / 64);
    const int32_t rbs = (nb + m->n - 1) / m->n;   // closure row blocks per device
    std::vector<hipEvent_t> ev(m->n, nullptr), ready(m->n, nullptr);
    int r = SPE_OK;
    for (int d = 0; d < m->n && !r; ++d) {
        if (hipSetDevice(P[d].device) != hipSuccess || hipEventCreateWithFlags(&ev[d], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ready[d], hipEventDisableTiming) != hipSuccess)
            r = set_error(SPE_EHIP, "FW closure events");
        if (!r) r = fw_init(m->graphs[d], P[d]);
    }
    FwBcast bc{m, P, ev, ready, m->gather == SPE_GATHER_RCCL};
    for (int32_t kb = 0; kb < nb && !r; ++kb) {
        const int own = kb / rbs;
        r = fw_pivot_owner(P[own], kb);
        if (!r) r = bc.rows(own, (int64_t)kb * 64, (int64_t)kb * 64 + 64, P[own].R ? (1 | 2) : 1);   // (R: triple builds)
        for (int d = 0; d < m->n && !r; ++d)
            r = fw_pivot_rows(P[d], kb, std::min(nb, d * rbs), std::min(nb, (d + 1) * rbs));
    }
    for (int d = 0; d < m->n && !r; ++d)
        r = bc.rows(d, (int64_t)std::min(nb, d * rbs) * 64, (int64_t)std::min(nb, (d + 1) * rbs) * 64, 1 | 4);
    for (int d = 0; d < m->n; ++d) {
        if (hipSetDevice(P[d].device) == hipSuccess && P[d].stream) {
            const hipError_t e = hipStreamSynchronize((hipStream_t)P[d].stream);
            if (!r && e != hipSuccess) r = hip_fail("FW closure sync", e);
        }
        if (ev[d]) (void)hipEventDestroy(ev[d]);
        if (ready[d]) (void)hipEventDestroy(ready[d]);
    }
    if (r) return r;
    for (auto& p : P) *p.done = true;
    if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return SPE_OK;
}

int multi_build(MultiDev* m, spe_build_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    double fw_s = 0.0;
    if (m->fw) {
        if (int r = fw_closure_multi(m, &fw_s)) return r;
    }
    // Every device builds its share chunk by chunk; the device finishing chunk k
    // last issues gather round k (the other devices are already building chunk
    // k + 1: the gather runs on the gather streams under the builds), then each
    // device builds the local remainder while the last rounds are in flight.
    const int32_t rounds = m->cb > 0 ? (m->cb + m->chunk - 1) / m->chunk : 0;
    std::vector<int> rc(m->n, SPE_OK);
    std::vector<std::string> err(m->n);
    std::vector<double> busy(m->n, 0.0);
    std::vector<int32_t> arrived(std::max(1, rounds), 0);
    std::mutex mu;
    int gather_rc = SPE_OK;
    std::string gather_err;
    std::vector<std::thread> th;
    for (int d = 0; d < m->n; ++d) {
        th.emplace_back([&, d]() {
            const auto s0 = std::chrono::steady_clock::now();
            for (int32_t k = 0; k < rounds; ++k) {
                const int32_t c0 = std::min(m->b1[d], m->b0[d] + k * m->chunk);
                const int32_t c1 = std::min(m->b1[d], c0 + m->chunk);
                if (c1 > c0 && rc[d] == SPE_OK) {
                    rc[d] = spe_table_build_blocks(m->parts[d], c0, c1, nullptr);
                    if (rc[d]) err[d] = spe_last_error();
                }
                std::lock_guard<std::mutex> lk(mu);
                if (++arrived[k] == m->n && gather_rc == SPE_OK) {
                    bool ok = true;
                    for (int e = 0; e < m->n; ++e) ok &= rc[e] == SPE_OK;
                    if (ok && (gather_rc = gather_round(m, k))) gather_err = spe_last_error();
                }
            }
            if (m->lparts[d] && rc[d] == SPE_OK) {
                rc[d] = spe_table_build(m->lparts[d], nullptr);
                if (rc[d]) err[d] = spe_last_error();
            }
            busy[d] = std::chrono::duration<double>(std::chrono::steady_clock::now() - s0).count();
        });
    }
    for (auto& x : th) x.join();
    for (int d = 0; d < m->n; ++d)
        if (rc[d]) return set_error(rc[d], "device " + std::to_string(m->devs[d]) + ": " + err[d]);
    if (gather_rc) return set_error(gather_rc, gather_err);
    const auto t1 = std::chrono::steady_clock::now();
    for (int d = 0; d < m->n; ++d) {
        if (hipSetDevice(m->devs[d]) != hipSuccess) return set_error(SPE_EHIP, "hipSetDevice");
        const hipError_t he = hipStreamSynchronize(m->streams[d]);
        if (he != hipSuccess) return hip_fail("gather sync", he);
    }
    const auto t2 = std::chrono::steady_clock::now();
    spe_build_stats s{};
    for (int d = 0; d < m->n; ++d)
        for (spe_table* p : {m->parts[d], m->lparts[d]}) {
            if (!p) continue;
            spe_build_stats q = SPE_STRUCT_INIT(spe_build_stats);
            spe_table_build_stats(p, &q);
            s.iterations += q.iterations;
            s.active_rounds += q.active_rounds;
            s.launches += q.launches;
            s.relaxed_lanes += q.relaxed_lanes;
            s.fallback_blocks += q.fallback_blocks;
            s.derived_sources += q.derived_sources;
        }
    s.seconds = std::chrono::duration<double>(t2 - t0).count();
    s.gather_seconds = std::chrono::duration<double>(t2 - t1).count();   // gather time not hidden by the builds
    s.build_wait_seconds = *std::max_element(busy.begin(), busy.end());
    s.n_devices = m->n;
    s.gather = m->gather;
    s.shared_blocks = std::min(m->S, m->nblk);
    s.local_blocks = m->nblk - std::min(m->S, m->nblk);
    m->stats = s;
    if (stats) *stats = s;
    m->built = true;
    return SPE_OK;
}

bool multi_built(const MultiDev* m) { return m->built; }

// The part table holding row block b's next hops / hop counts, and the last
// block of that table's run: a share's part, or the home device's local part.
static spe_table* part_of(const MultiDev* m, int32_t b, int32_t* run_end) {
    if (b >= m->S) {
        *run_end = m->nblk;
        return m->lparts[0];
    }
    const int d = b / m->cb;
    *run_end = m->b1[d];
    return m->parts[d];
}

int multi_get(const MultiDev* m, int32_t s_slot, int32_t t_slot, spe_entry* out) {
    if (s_slot < 0 || s_slot >= m->A || t_slot < 0 || t_slot >= m->A) return set_error(SPE_EINVAL, "slot out of range");
    int32_t e = 0;
    return spe_table_get(part_of(m, s_slot / kWave, &e), s_slot, t_slot, out);
}

int multi_source_tree(MultiDev* m, int32_t s_slot, int32_t* parent) {
    if (s_slot < 0 || s_slot >= m->A) return set_error(SPE_EINVAL, "slot out of range");
    int32_t e = 0;
    return spe_table_source_tree(part_of(m, s_slot / kWave, &e), s_slot, parent);
}

int multi_download(const MultiDev* m, int32_t row_begin, int32_t row_end, double* latency, double* reliability,
                   int32_t* next_hop, int32_t* hops) {
    if (row_begin < 0 || row_end > m->A || row_begin > row_end) return set_error(SPE_EINVAL, "row range out of bounds");
    for (int32_t r0 = row_begin; r0 < row_end;) {
        int32_t be = 0;
        spe_table* p = part_of(m, r0 / kWave, &be);
        const int32_t r1 = std::min(row_end, be * kWave);
        const size_t off = (size_t)(r0 - row_begin) * m->A;
        int rc = spe_table_download(p, r0, r1, latency ? latency + off : nullptr,
                                    reliability ? reliability + off : nullptr, next_hop ? next_hop + off : nullptr,
                                    hops ? hops + off : nullptr);
        if (rc) return rc;
        r0 = r1;
    }
    return SPE_OK;
}

int multi_lookup(const MultiDev* m, int32_t replica, const int32_t* d_pairs, int64_t q, double* d_latency,
                 double* d_reliability, uint8_t* d_ok, void* stream) {
    if (replica < 0 || replica >= m->n) return set_error(SPE_EINVAL, "replica out of range");
    return lookup_on_replica(m->devs[replica], m->replica[replica], m->A, m->nblk, d_pairs, q, d_latency, d_reliability,
                             d_ok, stream);
}

int multi_replica_device(const MultiDev* m, int32_t replica, int32_t* device) {
    if (replica < 0 || replica >= m->n) return set_error(SPE_EINVAL, "replica out of range");
    *device = m->devs[replica];
    return SPE_OK;
}

int multi_min_latency(const MultiDev* m, double* out) {
    double best = 0.0;
    std::vector<spe_table*> ts(m->parts);
    ts.push_back(m->lparts[0]);
    for (spe_table* p : ts) {
        if (!p) continue;
        double v = 0.0;
        if (int r = spe_table_min_latency(p, &v)) return r;
        if (v > 0 && (best == 0.0 || v < best)) best = v;   // 0 = the reference's "unset"
    }
    *out = best;
    return SPE_OK;
}

int multi_layout(const MultiDev* m, spe_table_layout* out) {
    spe_table_layout p = SPE_STRUCT_INIT(spe_table_layout);
    for (spe_table* x : {m->parts[0], m->lparts[0]})
        if (x) {
            spe_table_layout_get(x, &p);
            break;
        }
    out->n_attached = m->A;
    out->block_begin = 0;
    out->block_end = m->nblk;
    out->elems = (int64_t)m->span * m->A * kWave;
    out->latrel = m->replica[0];
    out->next_hop = nullptr;
    out->hops = nullptr;
    out->groups_per_launch = p.groups_per_launch;
    out->engine = p.engine;
    out->lanes_per_group = p.lanes_per_group;
    out->relax_kernel = p.relax_kernel;
    out->contracted_vertices = p.contracted_vertices;
    out->shared_sources = p.shared_sources;
    out->host_reads = 0;
    out->host_prefault = -1;
    out->host_prefault_s = 0.0;   // multi-device gets route to the part that built the row (copies)
    out->n_devices = m->n;
    out->device = m->devs[0];
    return SPE_OK;
}

int multi_profile_enable(MultiDev* m, int32_t enable) {
    for (int d = 0; d < m->n; ++d)
        for (spe_table* p : {m->parts[d], m->lparts[d]})
            if (p)
                if (int r = spe_table_profile_enable(p, enable)) return r;
    return SPE_OK;
}

int multi_profile_get(const MultiDev* m, spe_kernel_profile* out) {
    *out = spe_kernel_profile{};
    for (int d = 0; d < m->n; ++d) {
        spe_kernel_profile dev{};   // one device: its parts run one after the other
        for (spe_table* p : {m->parts[d], m->lparts[d]}) {
            if (!p) continue;
            spe_kernel_profile k{};
            spe_table_profile_get(p, &k);
            for (int i = 0; i < SPE_K_COUNT; ++i) {
                dev.ms[i] += k.ms[i];
                dev.launches[i] += k.launches[i];
            }
        }
        for (int i = 0; i < SPE_K_COUNT; ++i) {
            out->ms[i] = std::max(out->ms[i], dev.ms[i]);   // the devices run concurrently: the slowest
            out->launches[i] += dev.launches[i];
        }
    }
    return SPE_OK;
}

}  // namespace spe

extern "C" int spe_device_split(int32_t n_attached, int32_t n_devices, double shared_fraction, int32_t* block_begin,
                                int32_t* block_end, int32_t* local_begin) {
    if (n_attached < 0 || n_devices < 1 || !block_begin || !block_end || !local_begin || shared_fraction < 0.0 ||
        shared_fraction > 1.0)
        return spe::set_error(SPE_EINVAL, "spe_device_split: bad arguments");
    const int32_t nblk = (n_attached + 63) / 64;
    if (shared_fraction >= 1.0) {
        *local_begin = nblk;
        return spe_device_shares(n_attached, n_devices, block_begin, block_end);
    }
    const int32_t cb = (int32_t)std::floor(shared_fraction * nblk / n_devices);
    const int32_t S = n_devices * cb;   // <= nblk: every share full, the remainder local
    for (int32_t d = 0; d < n_devices; ++d) {
        block_begin[d] = d * cb;
        block_end[d] = (d + 1) * cb;
    }
    *local_begin = S;
    return SPE_OK;
}

extern "C" int spe_device_shares(int32_t n_attached, int32_t n_devices, int32_t* block_begin, int32_t* block_end) {
    if (n_attached < 0 || n_devices < 1 || !block_begin || !block_end)
        return spe::set_error(SPE_EINVAL, "spe_device_shares: bad arguments");
    const int32_t nblk = (n_attached + 63) / 64;
    const int32_t cb = (nblk + n_devices - 1) / n_devices;
    for (int32_t d = 0; d < n_devices; ++d) {
        block_begin[d] = std::min(nblk, d * cb);
        block_end[d] = std::min(nblk, (d + 1) * cb);
    }
    return SPE_OK;
}
