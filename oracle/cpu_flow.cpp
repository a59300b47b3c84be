// cpu_flow.cpp — TEST INFRASTRUCTURE (oracle/): a plain C++ / OpenMP restatement
// of the reference's CPU forward pass, used by tests/ (pinned against the numpy
// oracle, oracle/flow_oracle.py) and by bench.py's cpu_baseline leg ONLY.  The
// product path never links or loads it.
//
// It restates FlowChain.forward (src/Chains.jl:168-184) over
//   RNVPCouplingLayer  src/affine/RNVP.jl:168-187   x_af = z_af .* exp.(s) .+ t, ldj = Σ_rows s
//   NICECouplingLayer  src/affine/NICE.jl:135-153   x_af = z_af .+ t,            ldj = 0
//   CouplingBlock      src/Blocks.jl:140-150        layer_1 then layer_2, ldj_1 .+ ldj_2
//   NormalizationLayer src/norm/Normalization.jl:79-92
// with the conditioner input vcat(θ, z)[axis_nn, :] (src/affine/RNVP.jl:174) and
// Flux's Dense σ.(W*x .+ b) (Flux 0.16, NNlib.fast_act: tanh_fast / sigmoid_fast),
// in Flux's unfused op order: every Dense is a (out × in)·(in × S) product over a
// block of S samples, then the broadcast bias add, then σ — what Flux does per
// batch with BLAS sgemm, here as cache-blocked loops the compiler vectorises over
// the S samples of a block, one block per OpenMP thread at a time.  T = float is the
// timed CPU proxy; T = double is checked against the numpy fp64 oracle.
//
// The chain arrives as a pre-order program (built by oracle/cpu_flow.py):
//   CHAIN  : [0, k, child_1 … child_k]
//   BLOCK  : [1, layer_1, layer_2]
//   RNVP   : [2, n_af, af… (z rows), n_nn, nn… (vcat(θ, z) rows), ns, {in, out, act, has_b}×ns, nt, {…}×nt]   (0-based indices)
//   NICE   : [3, …as RNVP with ns = 0…]
//   NORM   : [4]                (x_min[d], x_max[d], α, β, ldj constant from the parameter stream)
// and the parameters as one stream of doubles in program order (per Dense: W
// column-major out×in, then b when present; per NORM: x_min, x_max, α, β, c).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include <omp.h>

namespace {

enum { ACT_ID = 0, ACT_RELU, ACT_TANH, ACT_SIGMOID, ACT_SOFTPLUS, ACT_LOGCOSH, ACT_LEAKY, ACT_ELU, ACT_SWISH };

constexpr int S = 128;  // samples per block (the vectorised dimension)

template <typename T>
inline T sigmoid_(T x) {
    const T t = std::exp(-std::fabs(x));
    return x >= T(0) ? T(1) / (T(1) + t) : t / (T(1) + t);
}

template <typename T>
inline T mad(T a, T b, T c);
template <>
inline float mad<float>(float a, float b, float c) { return std::fma(a, b, c); }
template <>
inline double mad<double>(double a, double b, double c) { return a * b + c; }

template <typename T>
inline T tanh_fast(T x) {  // NNlib.tanh_fast, Float32 coefficients (evalpoly with muladd)
    const T x2 = x * x;
    T n = T(1.587199e-8);  // evalpoly's leading coefficient (the oracle keeps it unrounded in fp64)
    n = mad(n, x2, T(2.2332108e-5f));
    n = mad(n, x2, T(0.0035974074f));
    n = mad(n, x2, T(0.1346604f));
    n = mad(n, x2, T(1.0f));
    T d = T(8.7767893e-7);
    d = mad(d, x2, T(0.0003453992f));
    d = mad(d, x2, T(0.026262015f));
    d = mad(d, x2, T(0.4679937f));
    d = mad(d, x2, T(1.0f));
    return x2 < T(66) ? x * (n / d) : (x > T(0) ? T(1) : (x < T(0) ? T(-1) : x));
}

template <typename T>
inline T softplus_(T x) { return std::log1p(std::exp(-std::fabs(x))) + (x > T(0) ? x : T(0)); }

template <typename T>
inline T act(int a, T x) {
    switch (a) {
        case ACT_RELU: return x > T(0) ? x : (x != x ? x : T(0));
        case ACT_TANH: return tanh_fast(x);
        case ACT_SIGMOID: return x > T(40) ? T(1) : (x < T(-80) ? T(0) : sigmoid_(x));
        case ACT_SOFTPLUS: return softplus_(x);
        case ACT_LOGCOSH: return (x + softplus_(T(-2) * x)) - T(0.6931471805599453);
        case ACT_LEAKY: return x > T(0) ? x : T(0.01) * x;
        case ACT_ELU: return x > T(0) ? x : std::expm1(x);
        case ACT_SWISH: return x * sigmoid_(x);
        default: return x;
    }
}

template <typename T>
struct Dense {
    int in, out, act, has_b;
    std::vector<T> W, b;  // W column-major (out × in)
};

template <typename T>
struct Node {
    int kind = 0;
    std::vector<int> children;
    std::vector<int> af, nn;
    std::vector<Dense<T>> s, t;
    std::vector<T> xmin, xmax;
    T alpha = 0, beta = 1, c = 0;
};

template <typename T>
struct Prog {
    std::vector<Node<T>> nodes;
    int d = 0, n = 0, maxw = 1;
    int root = 0;
};

template <typename T>
int parse(Prog<T>& P, const int32_t*& p, const double*& q) {
    const int id = (int)P.nodes.size();
    P.nodes.emplace_back();
    const int kind = *p++;
    P.nodes[id].kind = kind;
    if (kind == 0) {
        const int k = *p++;
        for (int i = 0; i < k; ++i) {
            const int c = parse(P, p, q);
            P.nodes[id].children.push_back(c);
        }
    } else if (kind == 1) {
        const int a = parse(P, p, q);
        const int b = parse(P, p, q);
        P.nodes[id].children = {a, b};
    } else if (kind == 2 || kind == 3) {
        Node<T> N;
        N.kind = kind;
        const int naf = *p++;
        for (int i = 0; i < naf; ++i) N.af.push_back(*p++);
        const int nnn = *p++;
        for (int i = 0; i < nnn; ++i) N.nn.push_back(*p++);
        for (int net = 0; net < 2; ++net) {
            const int nd = *p++;
            for (int k = 0; k < nd; ++k) {
                Dense<T> D;
                D.in = *p++;
                D.out = *p++;
                D.act = *p++;
                D.has_b = *p++;
                D.W.resize((size_t)D.in * D.out);
                for (auto& w : D.W) w = (T)*q++;
                if (D.has_b) {
                    D.b.resize(D.out);
                    for (auto& v : D.b) v = (T)*q++;
                }
                if (D.out > P.maxw) P.maxw = D.out;
                if (D.in > P.maxw) P.maxw = D.in;
                (net == 0 ? N.s : N.t).push_back(std::move(D));
            }
        }
        P.nodes[id] = std::move(N);
    } else {  // NORM
        Node<T>& N = P.nodes[id];
        N.xmin.resize(P.d);
        N.xmax.resize(P.d);
        for (auto& v : N.xmin) v = (T)*q++;
        for (auto& v : N.xmax) v = (T)*q++;
        N.alpha = (T)*q++;
        N.beta = (T)*q++;
        N.c = (T)*q++;
    }
    return id;
}

// one Dense over a block: Y[o][j] = σ(Σ_k W[o,k] X[k][j] + b[o]), j < S.
// Register-blocked like a BLAS micro-kernel: 4 outputs × 32 samples of
// accumulators per pass over k (each loaded x vector feeds 4 FMAs).
constexpr int JB = 64, OB = 4;

template <typename T>
void dense(const Dense<T>& D, const T* X, T* Y) {
    for (int o0 = 0; o0 < D.out; o0 += OB) {
        const int no = D.out - o0 < OB ? D.out - o0 : OB;
        for (int j0 = 0; j0 < S; j0 += JB) {
            T acc[OB][JB];
            for (int r = 0; r < OB; ++r)
                for (int j = 0; j < JB; ++j) acc[r][j] = T(0);
            for (int k = 0; k < D.in; ++k) {
                const T* x = X + (size_t)k * S + j0;
                const T* wk = D.W.data() + (size_t)k * D.out + o0;
                T w[OB];
                for (int r = 0; r < OB; ++r) w[r] = r < no ? wk[r] : T(0);
                for (int r = 0; r < OB; ++r)
#pragma omp simd
                    for (int j = 0; j < JB; ++j) acc[r][j] += w[r] * x[j];
            }
            for (int r = 0; r < no; ++r) {
                const int o = o0 + r;
                T* y = Y + (size_t)o * S + j0;
                const T b = D.has_b ? D.b[o] : T(0);
                if (D.has_b)
                    for (int j = 0; j < JB; ++j) acc[r][j] = acc[r][j] + b;
                if (D.act == ACT_RELU) {
                    for (int j = 0; j < JB; ++j) y[j] = acc[r][j] > T(0) ? acc[r][j] : T(0);
                } else if (D.act == ACT_ID) {
                    for (int j = 0; j < JB; ++j) y[j] = acc[r][j];
                } else {
                    for (int j = 0; j < JB; ++j) y[j] = act(D.act, acc[r][j]);
                }
            }
        }
    }
}

template <typename T>
struct Work {
    std::vector<T> a, b, in, sv, tv;
};

template <typename T>
void mlp(const std::vector<Dense<T>>& net, const T* X, T* out, Work<T>& w) {
    const T* cur = X;
    for (size_t k = 0; k < net.size(); ++k) {
        T* dst = (k + 1 == net.size()) ? out : ((k & 1) ? w.b.data() : w.a.data());
        dense(net[k], cur, dst);
        cur = dst;
    }
}

// z: state [d][S], th: [n][S], ldj: [S]
template <typename T>
void fwd(const Prog<T>& P, int id, T* z, const T* th, T* ldj, Work<T>& w) {
    const Node<T>& N = P.nodes[id];
    if (N.kind == 0 || N.kind == 1) {  // chain / block: ldj = ldj_1; ldj = ldj .+ ldj_i
        T li[S];
        fwd(P, N.children[0], z, th, ldj, w);
        for (size_t c = 1; c < N.children.size(); ++c) {
            fwd(P, N.children[c], z, th, li, w);
            for (int j = 0; j < S; ++j) ldj[j] = ldj[j] + li[j];
        }
        return;
    }
    if (N.kind == 4) {  // NormalizationLayer: (x_diff·z − α·x_max + β·x_min) / δ
        const T delta = N.beta - N.alpha;
        for (int i = 0; i < P.d; ++i) {
            const T xd = N.xmax[i] - N.xmin[i], am = N.alpha * N.xmax[i], bm = N.beta * N.xmin[i];
            T* zi = z + (size_t)i * S;
            for (int j = 0; j < S; ++j) zi[j] = ((xd * zi[j] - am) + bm) / delta;
        }
        for (int j = 0; j < S; ++j) ldj[j] = N.c;
        return;
    }
    // conditioner input vcat(θ, z)[axis_nn]
    for (size_t f = 0; f < N.nn.size(); ++f) {
        const int slot = N.nn[f];
        const T* src = slot < P.n ? th + (size_t)slot * S : z + (size_t)(slot - P.n) * S;
        std::memcpy(w.in.data() + f * S, src, sizeof(T) * S);
    }
    mlp(N.t, w.in.data(), w.tv.data(), w);
    const int naf = (int)N.af.size();
    if (N.kind == 2) {
        mlp(N.s, w.in.data(), w.sv.data(), w);
        for (int j = 0; j < S; ++j) ldj[j] = T(0);
        for (int k = 0; k < naf; ++k) {  // Σ_rows s in row order
            const T* s = w.sv.data() + (size_t)k * S;
            for (int j = 0; j < S; ++j) ldj[j] = ldj[j] + s[j];
        }
        for (int k = 0; k < naf; ++k) {
            T* zk = z + (size_t)N.af[k] * S;
            const T* s = w.sv.data() + (size_t)k * S;
            const T* t = w.tv.data() + (size_t)k * S;
            for (int j = 0; j < S; ++j) zk[j] = zk[j] * std::exp(s[j]) + t[j];
        }
    } else {
        for (int j = 0; j < S; ++j) ldj[j] = T(0);
        for (int k = 0; k < naf; ++k) {
            T* zk = z + (size_t)N.af[k] * S;
            const T* t = w.tv.data() + (size_t)k * S;
            for (int j = 0; j < S; ++j) zk[j] = zk[j] + t[j];
        }
    }
}

template <typename T>
int run(const int32_t* prog, const double* params, int d, int n, const T* z, const T* theta, T* x, T* ldj,
        int64_t B, int threads) {
    Prog<T> P;
    P.d = d;
    P.n = n;
    const int32_t* p = prog;
    const double* q = params;
    P.root = parse(P, p, q);
    const int64_t nblk = (B + S - 1) / S;
    const int W = P.maxw > d + n ? P.maxw : d + n;
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
    {
        Work<T> w;
        w.a.resize((size_t)W * S);
        w.b.resize((size_t)W * S);
        w.in.resize((size_t)W * S);
        w.sv.resize((size_t)W * S);
        w.tv.resize((size_t)W * S);
        std::vector<T> zs((size_t)d * S), ts((size_t)(n > 0 ? n : 1) * S), ls(S);
#pragma omp for schedule(static)
        for (int64_t blk = 0; blk < nblk; ++blk) {
            const int64_t j0 = blk * S;
            const int cnt = (int)((B - j0) < S ? (B - j0) : S);
            for (int j = 0; j < S; ++j) {  // (d, B) column-major → [d][S]
                const int64_t s = j0 + (j < cnt ? j : cnt - 1);
                for (int i = 0; i < d; ++i) zs[(size_t)i * S + j] = z[s * d + i];
                for (int i = 0; i < n; ++i) ts[(size_t)i * S + j] = theta[s * n + i];
            }
            fwd(P, P.root, zs.data(), ts.data(), ls.data(), w);
            for (int j = 0; j < cnt; ++j) {
                for (int i = 0; i < d; ++i) x[(j0 + j) * d + i] = zs[(size_t)i * S + j];
                ldj[j0 + j] = ls[j];
            }
        }
    }
    return 0;
}

}  // namespace

extern "C" {

int cpu_flow_forward_f32(const int32_t* prog, const double* params, int d, int n, const float* z,
                         const float* theta, float* x, float* ldj, int64_t B, int threads) {
    return run<float>(prog, params, d, n, z, theta, x, ldj, B, threads);
}

int cpu_flow_forward_f64(const int32_t* prog, const double* params, int d, int n, const double* z,
                         const double* theta, double* x, double* ldj, int64_t B, int threads) {
    return run<double>(prog, params, d, n, z, theta, x, ldj, B, threads);
}

int cpu_flow_max_threads(void) { return omp_get_max_threads(); }
}
