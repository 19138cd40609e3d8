// `tsp_search` — exact search of ONE instance on 1..G MI355X GPUs (K2), with
// the extension inputs the reference's CLI cannot express (BASELINE.json
// configs 1, 4 and 5):
//
//   tsp_search --random N [--seed S] [--clustered K]     uniform (or K Gaussian
//                                                         clusters) cities in [0,1000)^2
//   tsp_search --cities FILE [--tsplib-round]            "id x y" lines, or a TSPLIB
//                                                         file with NODE_COORD_SECTION
//   tsp_search --matrix FILE                              n, then n*n distances (all
//                                                         integers -> integer mode)
//   tsp_search --tsplib FILE                              a TSPLIB instance (EUC_2D,
//                                                         CEIL_2D, ATT, GEO or EXPLICIT
//                                                         weights: integer mode), e.g.
//                                                         tests/golden/tsplib/gr17.tsp
//   options: --gpus G (shard g on device g mod visible devices)  --rccl (the RCCL
//            exchange even for G = 1)  --solver auto|wide|k1|k2|enum  --verify (n <= 20: K1 too)
//   (enum: every tour enumerated on one GPU, BASELINE config 2)
//   auto = K1-wide (the DP with every CU on each layer) up to 25 cities on one
//   GPU, else K2 over the GPUs.
//
// City distances are the reference's computeDistanceMatrix (assignment2.h:
// 184-200, glibc pow/sqrt, f64); --tsplib-round uses TSPLIB's EUC_2D nint()
// instead (integer mode).  The answer is the reference's: the optimal
// left-fold cost and the DP's tie-broken tour.
//
// Multi-GPU: one host thread and one context per shard; shard g of G seeds
// the prefixes p = g mod G; after every few steps the incumbent word is
// combined in place with an RCCL all-reduce MIN (uint64, over xGMI; through
// the host when shards share a device), and the final optimum is that
// all-reduce's result; the optimal records of all shards then go through
// tspgpu_select_tour.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <barrier>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "tspgpu.h"

namespace {

[[noreturn]] void die(const char *msg)
{
    std::fprintf(stderr, "tsp_search: %s\n", msg);
    std::exit(2);
}

uint64_t splitmix(uint64_t &s)
{
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
double uniform(uint64_t &s) { return (double)(splitmix(s) >> 11) * 0x1p-53; }

struct Instance {
    int n = 0;
    int dtype = TSPGPU_F64;
    std::vector<double> d;
    std::vector<int32_t> di;
    std::string what;
};

std::vector<tspgpu_city> random_cities(int n, uint64_t seed, int clusters)
{
    std::vector<tspgpu_city> c(n);
    uint64_t s = seed;
    std::vector<double> cx(clusters > 0 ? clusters : 0), cy(cx.size());
    for (size_t k = 0; k < cx.size(); ++k) {
        cx[k] = 100.0 + 800.0 * uniform(s);
        cy[k] = 100.0 + 800.0 * uniform(s);
    }
    for (int i = 0; i < n; ++i) {
        c[i].id = i;
        if (clusters > 0) {
            // Box-Muller, sigma = 0.05 * grid
            const int k = i % clusters;
            const double u1 = 1.0 - uniform(s), u2 = uniform(s);
            const double r = std::sqrt(-2.0 * std::log(u1)) * 50.0;
            c[i].x = cx[k] + r * std::cos(2.0 * M_PI * u2);
            c[i].y = cy[k] + r * std::sin(2.0 * M_PI * u2);
        } else {
            c[i].x = 1000.0 * uniform(s);
            c[i].y = 1000.0 * uniform(s);
        }
    }
    return c;
}

std::vector<tspgpu_city> read_cities(const char *path)
{
    std::ifstream f(path);
    if (!f) die("cannot open the cities file");
    std::vector<tspgpu_city> c;
    std::string line;
    bool tsplib = false, in_coords = false;
    while (std::getline(f, line)) {
        if (line.find("NODE_COORD_SECTION") != std::string::npos) {
            tsplib = in_coords = true;
            continue;
        }
        if (line.find("EOF") == 0) break;
        if (tsplib && !in_coords) continue;
        if (!tsplib && (line.find(':') != std::string::npos)) {  // a TSPLIB header line
            tsplib = true;
            continue;
        }
        std::istringstream ss(line);
        tspgpu_city t{};
        double id;
        if (ss >> id >> t.x >> t.y) {
            t.id = (int)c.size();
            c.push_back(t);
        }
    }
    if (c.size() < 3) die("need at least 3 cities");
    return c;
}

Instance from_cities(const std::vector<tspgpu_city> &c, bool tsplib_round)
{
    Instance in;
    in.n = (int)c.size();
    in.d.resize((size_t)in.n * in.n);
    if (int rc = tspgpu_distance_matrix(c.data(), in.n, 1, in.d.data())) die(tspgpu_strerror(rc));
    if (tsplib_round) {
        in.dtype = TSPGPU_I32;
        in.di.resize(in.d.size());
        for (size_t i = 0; i < in.d.size(); ++i) in.di[i] = (int32_t)std::lround(in.d[i]);  // TSPLIB nint
    }
    return in;
}

// TSPLIB95 instance -> integer matrix (the same reader as tspgpu.read_tsplib):
// EDGE_WEIGHT_TYPE EUC_2D / CEIL_2D / ATT / GEO (TSPLIB's integer distance
// functions; GEO degrees truncated like Concorde) or EXPLICIT with
// EDGE_WEIGHT_FORMAT FULL_MATRIX / UPPER_ROW / LOWER_ROW / UPPER_DIAG_ROW /
// LOWER_DIAG_ROW.
Instance read_tsplib(const char *path)
{
    std::ifstream f(path);
    if (!f) die("cannot open the TSPLIB file");
    std::string line, kind = "EUC_2D", fmt = "FULL_MATRIX", name = path, section;
    int n = 0;
    std::vector<double> xs, ys;
    std::vector<long> w;
    auto trim = [](std::string t) {
        const size_t a = t.find_first_not_of(" \t\r"), b = t.find_last_not_of(" \t\r");
        return a == std::string::npos ? std::string() : t.substr(a, b - a + 1);
    };
    while (std::getline(f, line)) {
        const std::string t = trim(line);
        if (t.empty()) continue;
        if (t == "EOF") break;
        if (t.rfind("NODE_COORD_SECTION", 0) == 0) { section = "coord"; continue; }
        if (t.rfind("EDGE_WEIGHT_SECTION", 0) == 0) { section = "weight"; continue; }
        const std::string first = t.substr(0, t.find_first_of(" \t:"));
        if (first.size() > 8 && first.compare(first.size() - 8, 8, "_SECTION") == 0) { section = "skip"; continue; }
        if (section.empty() && t.find(':') != std::string::npos) {
            const std::string k = trim(t.substr(0, t.find(':'))), v = trim(t.substr(t.find(':') + 1));
            if (k == "DIMENSION") n = std::atoi(v.c_str());
            else if (k == "EDGE_WEIGHT_TYPE") kind = v;
            else if (k == "EDGE_WEIGHT_FORMAT") fmt = v;
            else if (k == "NAME") name = v;
            continue;
        }
        std::istringstream ss(t);
        if (section == "coord") {
            double id, x, y;
            if (ss >> id >> x >> y) xs.push_back(x), ys.push_back(y);
        } else if (section == "weight") {
            double v;
            while (ss >> v) w.push_back((long)v);
        }
    }
    if (n < 3) die("TSPLIB: DIMENSION must be >= 3");
    Instance in;
    in.n = n;
    in.dtype = TSPGPU_I32;
    in.di.assign((size_t)n * n, 0);
    in.what = name;
    if (kind == "EXPLICIT") {
        size_t k = 0;
        for (int i = 0; i < n; ++i) {
            int j0 = 0, j1 = n;  // columns of row i in the file
            if (fmt == "UPPER_ROW") j0 = i + 1;
            else if (fmt == "LOWER_ROW") j1 = i;
            else if (fmt == "UPPER_DIAG_ROW") j0 = i;
            else if (fmt == "LOWER_DIAG_ROW") j1 = i + 1;
            else if (fmt != "FULL_MATRIX") die("TSPLIB: EDGE_WEIGHT_FORMAT not supported");
            for (int j = j0; j < j1; ++j) {
                if (k >= w.size()) die("TSPLIB: EDGE_WEIGHT_SECTION too short");
                in.di[(size_t)i * n + j] = (int32_t)w[k++];
                if (fmt != "FULL_MATRIX") in.di[(size_t)j * n + i] = (int32_t)w[k - 1];
            }
        }
        return in;
    }
    if ((int)xs.size() != n) die("TSPLIB: NODE_COORD_SECTION does not hold DIMENSION cities");
    auto geo = [](double v) {
        const double deg = (double)(long)v;
        return 3.141592 * (deg + 5.0 * (v - deg) / 3.0) / 180.0;
    };
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            if (i == j) continue;
            const double dx = xs[i] - xs[j], dy = ys[i] - ys[j];
            long v;
            if (kind == "GEO") {
                const double q1 = std::cos(geo(ys[i]) - geo(ys[j])), q2 = std::cos(geo(xs[i]) - geo(xs[j])),
                             q3 = std::cos(geo(xs[i]) + geo(xs[j]));
                v = (long)(6378.388 * std::acos(0.5 * ((1.0 + q1) * q2 - (1.0 - q1) * q3)) + 1.0);
            } else if (kind == "ATT") {
                const double r = std::sqrt((dx * dx + dy * dy) / 10.0);
                const long t = (long)(r + 0.5);
                v = t < r ? t + 1 : t;
            } else if (kind == "CEIL_2D") {
                v = (long)std::ceil(std::sqrt(dx * dx + dy * dy));
            } else if (kind == "EUC_2D") {
                v = (long)(std::sqrt(dx * dx + dy * dy) + 0.5);
            } else {
                die("TSPLIB: EDGE_WEIGHT_TYPE not supported");
            }
            in.di[(size_t)i * n + j] = (int32_t)v;
        }
    return in;
}

Instance read_matrix(const char *path)
{
    std::ifstream f(path);
    if (!f) die("cannot open the matrix file");
    Instance in;
    if (!(f >> in.n) || in.n < 3) die("matrix file: first token must be n >= 3");
    std::vector<std::string> tok((size_t)in.n * in.n);
    bool integral = true;
    for (auto &t : tok) {
        if (!(f >> t)) die("matrix file: fewer than n*n entries");
        if (t.find_first_of(".eE") != std::string::npos) integral = false;
    }
    if (integral) {
        in.dtype = TSPGPU_I32;
        in.di.resize(tok.size());
        for (size_t i = 0; i < tok.size(); ++i) in.di[i] = (int32_t)std::strtol(tok[i].c_str(), nullptr, 10);
    } else {
        in.d.resize(tok.size());
        for (size_t i = 0; i < tok.size(); ++i) in.d[i] = std::strtod(tok[i].c_str(), nullptr);
    }
    return in;
}

const void *dist_ptr(const Instance &in) { return in.dtype == TSPGPU_F64 ? (const void *)in.d.data() : in.di.data(); }

struct Result {
    double cost = 0.0;
    std::vector<int32_t> tour;
    uint64_t nodes = 0;
    double kernel_ms = 0.0;
    int rounds = 0;
    const char *exchange = "none";  // how the shards' incumbents were combined (K2)
    int tie = 0;      // K2 over shards: the winner came from the device tie keys (no record read)
    int chained = 0;  // K2 over shards: every shard ran as one device chain
};

// K2 over G shards of this process, shard g on device g mod (visible
// devices).  Each shard runs as ONE device chain (tspgpu_search_chain: every
// frontier level enqueued back to back, one synchronisation) with the
// incumbent exchanged between levels IN THE STREAM: an RCCL all-reduce MIN
// (uint64, over xGMI) enqueued every kChainExchangeLevels levels, no host
// round trip.  A shard too large to chain runs step by step, with the same
// all-reduce every `every` steps.  RCCL needs every shard on its own device
// (also G = 1 with force_rccl: a one-rank communicator); shards that share a
// device (a rehearsal on a smaller box) exchange through the host between
// steps instead.  The winner: after the last exchange the
// incumbent is the optimum on every shard; each shard reads its device tie
// slot at it, then an all-reduce MIN of w0 (and of w1 among the holders of
// that w0) picks the least key, certified once (tspgpu_tie_tour).  Only when
// that certificate cannot be given are the optimal records read and passed
// to tspgpu_select_tour.
constexpr int kChainExchangeLevels = 2;

struct ChainHook {
    ncclComm_t comm;
    int rc;
};

void chain_exchange(void *user, void *stream, void *word)
{
    auto *h = static_cast<ChainHook *>(user);
    if (ncclAllReduce(word, word, 1, ncclUint64, ncclMin, h->comm, (hipStream_t)stream) != ncclSuccess) h->rc = -EIO;
}

int search_multi(const Instance &in, int G, bool force_rccl, int exchange_every, Result &res)
{
    int ndev = tspgpu_device_count();
    if (ndev < 1) ndev = 1;
    const bool shared = G > ndev;
    const bool rccl = (G > 1 || force_rccl) && !shared;
    if (force_rccl && shared) die("--rccl needs one GPU per shard (RCCL takes one rank per device)");
    std::vector<ncclComm_t> comms(rccl ? G : 0);
    std::vector<int> devs(G);
    for (int g = 0; g < G; ++g) devs[g] = g % ndev;
    if (rccl && ncclCommInitAll(comms.data(), G, devs.data()) != ncclSuccess) die("RCCL initialisation failed");
    std::atomic<uint64_t> host_min{~0ull};
    res.exchange = rccl ? "rccl" : (G > 1 ? "host" : "none");
    double ub = 0.0;
    if (int rc = tspgpu_heuristic_tour(dist_ptr(in), in.dtype, in.n, &ub, nullptr)) return rc;
    std::vector<int> rcs(G, 0);
    std::vector<std::vector<tspgpu_tour_record>> recs(G);
    std::vector<uint64_t> nodes(G, 0), opt(G, 0);
    std::vector<double> ms(G, 0.0);
    std::vector<int> rounds(G, 0), chained(G, 0);
    std::vector<tspgpu_tie_slot> slots(G);
    std::atomic<int> busy{0}, failed{0};
    // the key exchange without RCCL: every shard's slot, combined by shard 0
    uint64_t key[3] = {~0ull, ~0ull, 0};  // least w0, least w1 of its holders, any overflow
    std::vector<int32_t> tie_tour(in.n + 1, 0);
    std::atomic<int> tie_ok{0};
    // frontier steps between two incumbent exchanges (--exchange-every, default 4)
    const int every = std::max(1, exchange_every);
    const bool two = in.n - 1 > 20;
    std::barrier sync(G);
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g) {
        th.emplace_back([&, g] {
            tspgpu_opts o;
            std::memset(&o, 0, sizeof o);
            o.device = devs[g];
            tspgpu_ctx *ctx = nullptr;
            tspgpu_search *s = nullptr;
            int rc = tspgpu_ctx_create(&o, &ctx);
            if (!rc) rc = tspgpu_search_create(ctx, dist_ptr(in), in.dtype, in.n, g, G, 0, &s);
            if (!rc) rc = tspgpu_search_set_bound(s, ub);
            hipStream_t st = ctx ? (hipStream_t)tspgpu_stream(ctx) : nullptr;
            // the key exchange's device words, allocated up front: a shard that
            // fails later still joins every collective (with neutral words)
            unsigned long long *dk = nullptr;
            if (!rc && rccl && hipMalloc((void **)&dk, 2 * sizeof(unsigned long long)) != hipSuccess) {
                dk = nullptr;
                rc = -ENOMEM;
            }
            // every shard must join every all-reduce: if one could not start, none goes on
            if (rc) failed.store(1);
            sync.arrive_and_wait();
            uint64_t pending = 0;
            if (!failed.load()) {
                ChainHook hk{rccl ? comms[g] : nullptr, 0};
                int done = 0;
                rc = tspgpu_search_chain(s, kChainExchangeLevels, rccl ? chain_exchange : nullptr, &hk, &done);
                if (!rc) rc = hk.rc;
                chained[g] = done;
                if (!rc && !done) {
                    rc = tspgpu_search_start(s);
                    pending = 1;
                }
            }
            for (; !failed.load();) {
                // up to `every` steps of this shard, then one exchange (the same
                // count on every shard, so the all-reduces pair up)
                for (int k = 0; k < every && !rc && pending; ++k) rc = tspgpu_search_step(s, &pending);
                busy.fetch_add(!rc && pending ? 1 : 0);
                // incumbent exchange: in-place RCCL all-reduce MIN on the device word
                void *w = s ? tspgpu_search_incumbent_device(s) : nullptr;
                if (rccl && w && ncclAllReduce(w, w, 1, ncclUint64, ncclMin, comms[g], st) != ncclSuccess) rc = -EIO;
                if (st) (void)hipStreamSynchronize(st);
                if (!rccl && G > 1) {
                    // shared devices: MIN of the words through the host (the
                    // word only ever decreases, and no search kernel is running)
                    uint64_t inc = ~0ull, nd = 0, nr = 0;
                    if (s && !tspgpu_search_counters(s, &inc, &nd, &nr)) {
                        uint64_t cur = host_min.load();
                        while (inc < cur && !host_min.compare_exchange_weak(cur, inc)) {
                        }
                    }
                    sync.arrive_and_wait();
                    const uint64_t m = host_min.load();
                    if (s && m < inc) {
                        double b = 0.0;
                        if (in.dtype == TSPGPU_F64)
                            std::memcpy(&b, &m, 8);
                        else
                            b = (double)(int32_t)(uint32_t)m;
                        if (int r = tspgpu_search_set_bound(s, b)) rc = r;
                    }
                }
                sync.arrive_and_wait();
                const bool more = busy.load() > 0;
                sync.arrive_and_wait();
                if (g == 0) busy.store(0);
                sync.arrive_and_wait();
                if (!more) break;
            }
            uint64_t inc = 0, rec = 0;
            if (!rc && failed.load()) rc = -EIO;
            if (!rc) rc = tspgpu_search_counters(s, &inc, &nodes[g], &rec);
            opt[g] = inc;  // identical on every shard after the last all-reduce
            // the winner: all-reduce MIN of the tie key (w0, then w1 among its holders)
            tspgpu_tie_slot &ts = slots[g];
            std::memset(&ts, 0, sizeof ts);
            if (!rc) rc = tspgpu_search_tie_slot(s, inc, &ts);
            if (rccl && !failed.load()) {
                // (failed is the same for every shard after the start barrier;
                // otherwise every shard has dk and joins both collectives, a
                // shard whose counters or tie slot failed with neutral words:
                // no key, "overflow" so nobody certifies)
                unsigned long long hk[2] = {!rc && ts.found ? ts.w0 : ~0ull, !rc && !ts.overflow ? 1ull : 0ull};
                (void)hipMemcpyAsync(dk, hk, sizeof hk, hipMemcpyHostToDevice, st);
                if (ncclAllReduce(dk, dk, 2, ncclUint64, ncclMin, comms[g], st) != ncclSuccess && !rc) rc = -EIO;
                (void)hipMemcpyAsync(hk, dk, sizeof hk, hipMemcpyDeviceToHost, st);
                (void)hipStreamSynchronize(st);
                const uint64_t W0 = hk[0];
                const bool clean = hk[1] == 1;
                unsigned long long h1 = !rc && ts.found && ts.w0 == W0 ? ts.w1 : ~0ull;
                if (two) {
                    (void)hipMemcpyAsync(dk, &h1, 8, hipMemcpyHostToDevice, st);
                    if (ncclAllReduce(dk, dk, 1, ncclUint64, ncclMin, comms[g], st) != ncclSuccess && !rc) rc = -EIO;
                    (void)hipMemcpyAsync(&h1, dk, 8, hipMemcpyDeviceToHost, st);
                    (void)hipStreamSynchronize(st);
                }
                if (g == 0) {
                    key[0] = W0;
                    key[1] = two ? h1 : 0;
                    key[2] = clean ? 0 : 1;
                }
            } else if (!rccl) {
                sync.arrive_and_wait();
                if (g == 0) {
                    for (int q = 0; q < G; ++q) {
                        if (slots[q].overflow) key[2] = 1;
                        if (slots[q].found && slots[q].w0 < key[0]) key[0] = slots[q].w0;
                    }
                    for (int q = 0; q < G && two; ++q)
                        if (slots[q].found && slots[q].w0 == key[0] && slots[q].w1 < key[1]) key[1] = slots[q].w1;
                    if (!two) key[1] = 0;
                }
            }
            sync.arrive_and_wait();
            // certified once (shard 0, its prefix DPs on its GPU), then every
            // shard knows whether its records are needed
            if (g == 0 && !rc && !key[2] && key[0] != ~0ull &&
                tspgpu_tie_tour_gpu(ctx, dist_ptr(in), in.dtype, in.n, key[0], key[1], opt[0], tie_tour.data()) == 0)
                tie_ok.store(1);
            sync.arrive_and_wait();
            if (!rc && !tie_ok.load()) {
                int cnt = 0;
                recs[g].resize(rec);
                rc = tspgpu_search_records(s, inc, recs[g].data(), (int)rec, &cnt);
                recs[g].resize(cnt);
            }
            if (s) tspgpu_search_timing(s, &ms[g], &rounds[g]);
            if (dk) (void)hipFree(dk);
            if (s) tspgpu_search_destroy(s);
            if (ctx) tspgpu_ctx_destroy(ctx);
            rcs[g] = rc;
        });
    }
    for (auto &t : th) t.join();
    for (auto &c : comms) ncclCommDestroy(c);
    for (int rc : rcs)
        if (rc) return rc;  // incl. -EOVERFLOW (too many tied optima: use --solver k1)
    res.tour.assign(in.n + 1, 0);
    res.tie = tie_ok.load();
    res.chained = 1;
    for (int g = 0; g < G; ++g) res.chained &= chained[g];
    if (res.tie) {
        res.tour = tie_tour;
    } else {
        std::vector<tspgpu_tour_record> all;
        for (auto &r : recs) all.insert(all.end(), r.begin(), r.end());
        if (int rc = tspgpu_select_tour(dist_ptr(in), in.dtype, in.n, all.data(), (int)all.size(), opt[0],
                                        res.tour.data()))
            return rc;
    }
    if (in.dtype == TSPGPU_F64)
        std::memcpy(&res.cost, &opt[0], 8);
    else
        res.cost = (double)(int32_t)(uint32_t)opt[0];
    for (int g = 0; g < G; ++g) {
        res.nodes += nodes[g];
        res.kernel_ms = std::max(res.kernel_ms, ms[g]);
        res.rounds = std::max(res.rounds, rounds[g]);
    }
    return 0;
}

int solve_k1(const Instance &in, Result &res)
{
    if (in.n > TSPGPU_MAX_CITIES) return -EINVAL;
    std::vector<double> d = in.d;
    if (in.dtype == TSPGPU_I32) d.assign(in.di.begin(), in.di.end());
    res.tour.assign(in.n + 1, -1);
    tspgpu_opts o;
    std::memset(&o, 0, sizeof o);
    return tspgpu_solve(d.data(), in.n, 1, &res.cost, res.tour.data(), &o);
}

// K1-wide: the DP with every CU on each layer (n <= 31); integers are exact as f64
int solve_wide(const Instance &in, Result &res)
{
    if (in.n > TSPGPU_WIDE_MAX_CITIES) return -EINVAL;
    std::vector<double> d = in.d;
    if (in.dtype == TSPGPU_I32) d.assign(in.di.begin(), in.di.end());
    res.tour.assign(in.n + 1, -1);
    tspgpu_opts o;
    std::memset(&o, 0, sizeof o);
    o.device = 0;
    tspgpu_ctx *ctx = nullptr;
    int rc = tspgpu_ctx_create(&o, &ctx);
    if (!rc) rc = tspgpu_solve_instance(ctx, d.data(), in.n, &res.cost, res.tour.data(), &res.kernel_ms);
    if (ctx) tspgpu_ctx_destroy(ctx);
    return rc;
}

// exhaustive enumeration of all (n-1)! tours on GPU 0 (K2 with the bound off)
int solve_enum(const Instance &in, Result &res)
{
    tspgpu_opts o;
    std::memset(&o, 0, sizeof o);
    tspgpu_ctx *ctx = nullptr;
    int rc = tspgpu_ctx_create(&o, &ctx);
    res.tour.assign(in.n + 1, -1);
    tspgpu_search_stats st;
    std::memset(&st, 0, sizeof st);
    if (!rc) rc = tspgpu_search_enumerate(ctx, dist_ptr(in), in.dtype, in.n, &res.cost, res.tour.data(), &st);
    res.nodes = st.nodes;
    res.kernel_ms = st.kernel_ms;
    res.rounds = st.rounds;
    if (ctx) tspgpu_ctx_destroy(ctx);
    return rc;
}

}  // namespace

int main(int argc, char **argv)
{
    Instance in;
    bool have = false, verify = false, tsplib_round = false, dump = false;
    int gpus = 1, random_n = 0, clusters = 0, exchange_every = 4;
    bool force_rccl = false;
    uint64_t seed = 1;
    std::string solver = "auto", cities_file, matrix_file, tsplib_file;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) die("missing value");
            return argv[++i];
        };
        if (a == "--random") random_n = std::atoi(next());
        else if (a == "--seed") seed = std::strtoull(next(), nullptr, 10);
        else if (a == "--clustered") clusters = std::atoi(next());
        else if (a == "--cities") cities_file = next();
        else if (a == "--matrix") matrix_file = next();
        else if (a == "--tsplib") tsplib_file = next();
        else if (a == "--tsplib-round") tsplib_round = true;
        else if (a == "--gpus") gpus = std::atoi(next());
        else if (a == "--exchange-every") exchange_every = std::atoi(next());  // frontier steps between exchanges
        else if (a == "--rccl") force_rccl = true;  // the RCCL exchange even on one GPU (one-rank communicator)
        else if (a == "--solver") solver = next();
        else if (a == "--verify") verify = true;
        else if (a == "--dump-matrix") dump = true;  // print the instance's matrix and exit (no GPU)
        else {
            std::fprintf(stderr, "usage: tsp_search (--random N [--seed S] [--clustered K] | --cities FILE "
                                 "[--tsplib-round] | --matrix FILE | --tsplib FILE) [--gpus G] [--rccl] [--exchange-every S] [--solver auto|wide|k1|k2|enum] [--verify]\n");
            return 1;
        }
    }
    if (random_n) {
        if (random_n < 3 || random_n > TSPGPU_SEARCH_MAX_CITIES) die("--random N needs 3 <= N <= 32");
        in = from_cities(random_cities(random_n, seed, clusters), tsplib_round);
        have = true;
    } else if (!cities_file.empty()) {
        in = from_cities(read_cities(cities_file.c_str()), tsplib_round);
        have = true;
    } else if (!matrix_file.empty()) {
        in = read_matrix(matrix_file.c_str());
        have = true;
    } else if (!tsplib_file.empty()) {
        in = read_tsplib(tsplib_file.c_str());
        have = true;
    }
    if (!have) die("no instance (--random, --cities, --matrix or --tsplib)");
    if (dump) {
        std::printf("%d\n", in.n);
        for (int i = 0; i < in.n; ++i) {
            for (int j = 0; j < in.n; ++j) {
                if (in.dtype == TSPGPU_I32)
                    std::printf(j ? " %d" : "%d", in.di[(size_t)i * in.n + j]);
                else
                    std::printf(j ? " %.17g" : "%.17g", in.d[(size_t)i * in.n + j]);
            }
            std::printf("\n");
        }
        return 0;
    }
    if (gpus < 1) gpus = 1;
    // auto: the DP over the whole GPU (K1-wide) up to 25 cities on one GPU,
    // else the search (K2) over all GPUs
    // (with the Lagrangian two-edge bound K2 overtakes the DP from ~25 cities:
    // n = 28 2.0-2.5 ms vs ~10 ms, n = 30 2.3-5.8 ms vs ~40 ms;
    // profiles/r02/k2_lagrange.log)
    if (solver == "auto") solver = (in.n <= 25 && gpus == 1 && !force_rccl) ? "wide" : "k2";
    if (solver != "k1" && solver != "k2" && solver != "wide" && solver != "enum")
        die("--solver must be auto, wide, k1, k2 or enum");

    Result res;
    const auto t0 = std::chrono::steady_clock::now();
    int rc = solver == "k1"     ? solve_k1(in, res)
             : solver == "wide" ? solve_wide(in, res)
             : solver == "enum" ? solve_enum(in, res)
                                : search_multi(in, gpus, force_rccl, exchange_every, res);
    if (rc == -EOVERFLOW && in.n <= TSPGPU_WIDE_MAX_CITIES) {
        // more tied optima than the record buffers hold (e.g. coincident cities):
        // the DP returns the same tour directly
        std::fprintf(stderr, "tsp_search: too many tied optimal tours to enumerate; answering with the DP\n");
        solver = "wide";
        rc = solve_wide(in, res);
    }
    const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (rc) {
        std::fprintf(stderr, "tsp_search: %s (%d)\n", tspgpu_strerror(rc), rc);
        return 3;
    }
    std::printf("cities %d  mode %s  solver %s  gpus %d\n", in.n, in.dtype == TSPGPU_F64 ? "f64" : "i32",
                solver.c_str(), solver == "k2" ? gpus : 1);
    std::printf("optimal cost %.17g (%f)\n", res.cost, res.cost);
    std::printf("tour");
    for (int t : res.tour) std::printf(" %d", t);
    std::printf("\n");
    if (solver == "k2" || solver == "enum")
        std::printf("search nodes %llu  rounds %d  kernel %.3f ms  %.3f Gnodes/s  wall %.3f ms  exchange %s\n",
                    (unsigned long long)res.nodes, res.rounds, res.kernel_ms,
                    res.kernel_ms > 0 ? res.nodes / res.kernel_ms / 1e6 : 0.0, wall, res.exchange);
    if (solver == "k2" && std::strcmp(res.exchange, "none") != 0)  // (the sharded driver)
        std::printf("winner %s  chained %d\n", res.tie ? "tie-key" : "records", res.chained);
    if (solver == "wide")
        std::printf("kernel %.3f ms  wall %.3f ms\n", res.kernel_ms, wall);
    else if (solver != "k2" && solver != "enum")
        std::printf("wall %.3f ms\n", wall);
    if (verify && in.n <= TSPGPU_MAX_CITIES && solver != "k1") {
        Result k1;
        if ((rc = solve_k1(in, k1))) {
            std::fprintf(stderr, "tsp_search: K1 check failed: %s\n", tspgpu_strerror(rc));
            return 3;
        }
        const bool same = k1.cost == res.cost && k1.tour == res.tour;
        std::printf("K1 check: %s\n", same ? "identical cost and tour" : "MISMATCH");
        if (!same) return 4;
    }
    return 0;
}
