// matnet.cpp — the input-aware selector of IA-SpGEMM, natively:
// the matrix features (GetInfo1/2/3), the 128x128 density images, and the
// forward pass of MatNet, the small Keras CNN the reference asks which
// algorithm to run (IA-SPGEMM-CPU_release/MatNet.py Pred, :24-96; the GPU
// program's variant GPU/MatNet.py).  The weights are the reference's own
// NetWeights/*.h5, exported once to flat float32 blobs
// (tools/matnet_export.py -> ia-spgemm_amd/data/matnet_<set>.bin).  Host code:
// it runs once per call of the CLIs, off the timed path, as in the reference.
#include "ias.h"
#include "ias_internal.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace ias;

// w[2l] = kernel, w[2l+1] = bias of layer l: conv2d_1..6, dense_1..4
struct ias_matnet {
    int32_t nf = 0, nc = 0;
    std::vector<float> w[20];
};

namespace {

constexpr int SIDE = IAS_IMAGE_SIDE;

// Host view of a CSR (a device matrix is copied; the copy is owned here).
struct Host {
    ias_csr h{};
    const ias_csr *m = nullptr;
    bool owned = false;
    ~Host() {
        if (owned) ias_csr_free(&h);
    }
    ias_status get(const ias_csr *A) {
        if (A->memory == IAS_MEMORY_DEVICE) {
            IAS_TRY(ias_csr_copy(A, &h, IAS_MEMORY_HOST, 0));
            owned = true;
            m = &h;
        } else {
            m = A;
        }
        return IAS_SUCCESS;
    }
};

// GetInfo1 (csr/common_csr.h:257-287): rows, cols, nnz, density, max / min /
// mean nnz per row, sample variance, coefficient of variation.  Products the
// reference forms in int (row*col) are formed in double here.
void info1(const ias_csr *A, double *f) {
    const int64_t m = A->rows;
    const int64_t *rp = A->row_ptr;
    const double mean = (double)A->nnz / (double)m;
    int64_t mx = m > 0 ? rp[1] - rp[0] : 0, mn = mx;
    double var = 0.0;
    for (int64_t i = 0; i < m; ++i) {
        const int64_t n = rp[i + 1] - rp[i];
        mx = std::max(mx, n);
        mn = std::min(mn, n);
        var += ((double)n - mean) * ((double)n - mean);
    }
    var = var / (double)(m - 1);
    f[0] = (double)A->rows;
    f[1] = (double)A->cols;
    f[2] = (double)A->nnz;
    f[3] = (double)A->nnz / ((double)A->rows * (double)A->cols);
    f[4] = (double)mx;
    f[5] = (double)mn;
    f[6] = mean;
    f[7] = var;
    f[8] = std::sqrt(var) / mean;
}

// GetInfo2 (dia/common_dia.h:222-233) of CSRtoDIA(A): the diagonal count as
// CSRtoDIA counts it (dia:32-49, every stored entry marks its diagonal).
void info2(const ias_csr *A, double *f) {
    std::vector<char> seen((size_t)(A->rows + A->cols), 0);
    int64_t nd = 0;
    for (int64_t i = 0; i < A->rows; ++i)
        for (int64_t p = A->row_ptr[i]; p < A->row_ptr[i + 1]; ++p) {
            const int64_t idx = (A->rows - i) + A->col[p];
            if (!seen[idx]) {
                seen[idx] = 1;
                ++nd;
            }
        }
    f[0] = (double)nd;
    f[1] = (double)nd / (double)(A->rows + A->cols - 1);
    f[2] = ((double)nd * (double)A->rows) / ((double)A->rows * (double)A->cols);
}

// GetInfo3 (ell/common_ell.h:222-229) of CSRtoELL(A): fill of the padded rows.
void info3(const ias_csr *A, double *f) {
    int64_t mx = 0;
    for (int64_t i = 0; i < A->rows; ++i) mx = std::max(mx, A->row_ptr[i + 1] - A->row_ptr[i]);
    f[0] = (double)A->nnz / ((double)A->rows * (double)mx);
}

// ---- MatNet layers (Keras semantics, channels-last, float32)
// Conv2D (kernel k x k x C x O, stride s, 'valid' or TF 'same' padding:
// the extra padding row/column goes to the bottom/right) + tanh.
void conv_tanh(const std::vector<float> &in, int H, int W, int C, const std::vector<float> &K,
               const std::vector<float> &b, int k, int s, bool same, int O, std::vector<float> &out, int &OH,
               int &OW) {
    int pt = 0, pl = 0;
    if (same) {
        OH = (H + s - 1) / s;
        OW = (W + s - 1) / s;
        pt = std::max((OH - 1) * s + k - H, 0) / 2;
        pl = std::max((OW - 1) * s + k - W, 0) / 2;
    } else {
        OH = (H - k) / s + 1;
        OW = (W - k) / s + 1;
    }
    out.assign((size_t)OH * OW * O, 0.0f);
    std::vector<float> acc((size_t)O);
    for (int y = 0; y < OH; ++y)
        for (int x = 0; x < OW; ++x) {
            std::fill(acc.begin(), acc.end(), 0.0f);
            for (int dy = 0; dy < k; ++dy) {
                const int iy = y * s + dy - pt;
                if (iy < 0 || iy >= H) continue;
                for (int dx = 0; dx < k; ++dx) {
                    const int ix = x * s + dx - pl;
                    if (ix < 0 || ix >= W) continue;
                    const float *pin = &in[((size_t)iy * W + ix) * C];
                    const float *pk = &K[(size_t)(dy * k + dx) * C * O];
                    for (int c = 0; c < C; ++c) {
                        const float v = pin[c];
                        const float *kk = pk + (size_t)c * O;
                        for (int o = 0; o < O; ++o) acc[o] += v * kk[o];
                    }
                }
            }
            float *po = &out[((size_t)y * OW + x) * O];
            for (int o = 0; o < O; ++o) po[o] = std::tanh(acc[o] + b[o]);
        }
}

// MaxPooling2D(2, 2), 'valid'
void maxpool2(const std::vector<float> &in, int H, int W, int C, std::vector<float> &out, int &OH, int &OW) {
    OH = H / 2;
    OW = W / 2;
    out.assign((size_t)OH * OW * C, 0.0f);
    for (int y = 0; y < OH; ++y)
        for (int x = 0; x < OW; ++x)
            for (int c = 0; c < C; ++c) {
                auto at = [&](int yy, int xx) { return in[((size_t)yy * W + xx) * C + c]; };
                out[((size_t)y * OW + x) * C + c] =
                    std::max(std::max(at(2 * y, 2 * x), at(2 * y, 2 * x + 1)),
                             std::max(at(2 * y + 1, 2 * x), at(2 * y + 1, 2 * x + 1)));
            }
}

// Dense (kernel n x m), optional tanh
void dense(const float *in, int n, const std::vector<float> &K, const std::vector<float> &b, int m, bool act,
           float *out) {
    for (int j = 0; j < m; ++j) {
        float acc = 0.0f;
        for (int i = 0; i < n; ++i) acc += in[i] * K[(size_t)i * m + j];
        acc += b[j];
        out[j] = act ? std::tanh(acc) : acc;
    }
}

// One image branch (MatNet.py:45-55): conv 3x3 valid, pool, conv 5x5/2 same,
// pool, conv 5x5/2 same, pool, flatten -> 4*4*16 = 256 values.
void branch(const ias_matnet &net, int l0, const std::vector<float> &img, float *flat) {
    std::vector<float> a, b;
    int H = SIDE, W = SIDE, h, w;
    conv_tanh(img, H, W, 1, net.w[2 * l0], net.w[2 * l0 + 1], 3, 1, false, 16, a, h, w);
    maxpool2(a, h, w, 16, b, H, W);
    conv_tanh(b, H, W, 16, net.w[2 * l0 + 2], net.w[2 * l0 + 3], 5, 2, true, 16, a, h, w);
    maxpool2(a, h, w, 16, b, H, W);
    conv_tanh(b, H, W, 16, net.w[2 * l0 + 4], net.w[2 * l0 + 5], 5, 2, true, 16, a, h, w);
    maxpool2(a, h, w, 16, b, H, W);
    std::copy(b.begin(), b.end(), flat);   // H = W = 4: 256 values, (row, col, channel) order
}

// MatNet.py:29-37: image = count * 255 / max(count), fed to Keras as float32.
std::vector<float> normalise(const int64_t *img) {
    int64_t mx = 0;
    for (int i = 0; i < SIDE * SIDE; ++i) mx = std::max(mx, img[i]);
    std::vector<float> out((size_t)SIDE * SIDE);
    for (int i = 0; i < SIDE * SIDE; ++i) out[i] = (float)((double)img[i] * 255.0 / (double)mx);
    return out;
}

// Directory of the weight blobs: $IAS_MATNET_DIR, else <dir of libias.so>/data.
std::string data_dir() {
    const char *e = getenv("IAS_MATNET_DIR");
    if (e && *e) return e;
    Dl_info info{};
    if (dladdr((void *)&ias_matnet_load, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        const size_t slash = p.rfind('/');
        return (slash == std::string::npos ? std::string(".") : p.substr(0, slash)) + "/data";
    }
    return "data";
}

}  // namespace

extern "C" ias_status ias_features(const ias_csr *A, const ias_csr *B, int32_t nfeatures, double *features) {
    if (!A || !B || !features || (nfeatures != 26 && nfeatures != 18)) return IAS_ERROR_INVALID_ARGUMENT;
    IAS_TRY(check_csr_host(A));
    IAS_TRY(check_csr_host(B));
    Host ha, hb;
    IAS_TRY(ha.get(A));
    IAS_TRY(hb.get(B));
    std::fill(features, features + nfeatures, 0.0);
    info1(ha.m, features);
    info1(hb.m, features + 9);
    if (nfeatures == 26) {
        info2(ha.m, features + 18);
        info2(hb.m, features + 21);
        info3(ha.m, features + 24);
        info3(hb.m, features + 25);
    }
    return IAS_SUCCESS;
}

// main.cpp:516-565 (and GPU/main.cu:276-343): every stored entry (i, j)
// increments the cells [i*128/rows .. + 128/rows] x [j*128/cols .. + 128/cols]
// (one cell when the side exceeds 128, the identity when it equals 128).
extern "C" ias_status ias_density_image(const ias_csr *A, int64_t *image) {
    if (!A || !image) return IAS_ERROR_INVALID_ARGUMENT;
    IAS_TRY(check_csr_host(A));
    Host ha;
    IAS_TRY(ha.get(A));
    const ias_csr *M = ha.m;
    std::fill(image, image + SIDE * SIDE, (int64_t)0);
    auto span = [](int64_t v, int64_t n, int64_t &s, int64_t &e) {
        if (n > SIDE) {
            s = e = v * SIDE / n;
        } else if (n < SIDE) {
            s = v * SIDE / n;
            e = s + SIDE / n;
        } else {
            s = e = v;
        }
    };
    for (int64_t i = 0; i < M->rows; ++i) {
        int64_t is, ie;
        span(i, M->rows, is, ie);
        for (int64_t p = M->row_ptr[i]; p < M->row_ptr[i + 1]; ++p) {
            int64_t js, je;
            span(M->col[p], M->cols, js, je);
            for (int64_t k = is; k <= ie; ++k)
                for (int64_t m = js; m <= je; ++m)
                    if (k < SIDE && m < SIDE) ++image[k * SIDE + m];
        }
    }
    return IAS_SUCCESS;
}

extern "C" ias_status ias_matnet_load(const char *weights, ias_matnet **net) {
    if (!weights || !net) return IAS_ERROR_INVALID_ARGUMENT;
    *net = nullptr;
    std::string path = weights;
    if (path == "intel" || path == "amd" || path == "p100") path = data_dir() + "/matnet_" + path + ".bin";
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) {
        set_last_error("cannot open MatNet weights %s", path.c_str());
        return IAS_ERROR_IO;
    }
    char magic[8];
    int32_t hdr[2];
    ias_matnet *n = new ias_matnet();
    bool ok = fread(magic, 1, 8, f) == 8 && !memcmp(magic, "IASMNET1", 8) && fread(hdr, 4, 2, f) == 2 &&
              hdr[0] > 0 && hdr[0] <= 64 && hdr[1] > 0 && hdr[1] <= 64;
    if (ok) {
        n->nf = hdr[0];
        n->nc = hdr[1];
        const size_t sizes[20] = {9 * 16, 16, 25 * 256, 16, 25 * 256, 16, 9 * 16, 16, 25 * 256, 16, 25 * 256, 16,
                                  (size_t)n->nf * n->nf, (size_t)n->nf, 256 * 32, 32, 256 * 32, 32,
                                  (size_t)(64 + n->nf) * n->nc, (size_t)n->nc};
        for (int i = 0; i < 20 && ok; ++i) {
            n->w[i].resize(sizes[i]);
            ok = fread(n->w[i].data(), sizeof(float), sizes[i], f) == sizes[i];
        }
        char extra;
        ok = ok && fread(&extra, 1, 1, f) == 0;
    }
    fclose(f);
    if (!ok) {
        delete n;
        set_last_error("%s is not a MatNet weight blob (tools/matnet_export.py)", path.c_str());
        return IAS_ERROR_FORMAT;
    }
    *net = n;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_matnet_free(ias_matnet *net) {
    delete net;
    return IAS_SUCCESS;
}

extern "C" ias_status ias_matnet_shape(const ias_matnet *net, int32_t *nfeatures, int32_t *nclasses) {
    if (!net) return IAS_ERROR_INVALID_ARGUMENT;
    if (nfeatures) *nfeatures = net->nf;
    if (nclasses) *nclasses = net->nc;
    return IAS_SUCCESS;
}

// MatNet.py:40-92: two image branches, Dense(nf, tanh) over the features,
// Dense(32, tanh) per branch, concatenate [image 1, image 2, features],
// Dense(nc) + softmax; the choice is the argmax (first maximum).
extern "C" ias_status ias_matnet_predict(const ias_matnet *net, const int64_t *image_a, const int64_t *image_b,
                                         const double *features, float *probs, int32_t *chosen) {
    if (!net || !image_a || !image_b || !features || !chosen) return IAS_ERROR_INVALID_ARGUMENT;
    const int nf = net->nf, nc = net->nc;
    std::vector<float> fa(256), fb(256), feat((size_t)nf), cat((size_t)(64 + nf)), z((size_t)nc);
    branch(*net, 0, normalise(image_a), fa.data());
    branch(*net, 3, normalise(image_b), fb.data());
    for (int i = 0; i < nf; ++i) feat[i] = (float)features[i];
    dense(fa.data(), 256, net->w[14], net->w[15], 32, true, cat.data());
    dense(fb.data(), 256, net->w[16], net->w[17], 32, true, cat.data() + 32);
    dense(feat.data(), nf, net->w[12], net->w[13], nf, true, cat.data() + 64);
    dense(cat.data(), 64 + nf, net->w[18], net->w[19], nc, false, z.data());
    int best = 0;
    for (int j = 1; j < nc; ++j)
        if (z[j] > z[best]) best = j;
    if (probs) {
        float s = 0.0f;
        for (int j = 0; j < nc; ++j) s += (probs[j] = std::exp(z[j] - z[best]));
        for (int j = 0; j < nc; ++j) probs[j] /= s;
    }
    *chosen = best;
    return IAS_SUCCESS;
}
