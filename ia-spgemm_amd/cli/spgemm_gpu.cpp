// spgemm-gpu — drop-in for IA-SPGEMM-GPU_release/main.cu (the `spgemm-gpu`
// program).  Reads one .mtx, asks MatNet (the reference's P100 weights, run
// natively) for its choice, and reports the GPU algorithms; the reference's
// Algorithm 1 (CUSP ESC, main.cu:467-505) and Algorithm 2 (cuSPARSE csrgemm,
// main.cu:508-523) are replaced by this engine's two output orders:
//   1 IAS row-wise hash, reference order (byte-identical to CSR_MUL_CSR)
//   2 IAS row-wise hash + per-row sort (sorted columns, as csrgemm emits)
// Usage: spgemm-gpu A.mtx [--aat] [--rand10] [--seed N] [--mtx-out C.mtx]
//                        [--gpus N | --devices d0,d1,...]
//   default C = A*A (the README's contract); --aat builds B = A^T on the
//   device, as main.cu:260-269 does with mkl_dcsrcsc; --rand10 replaces
//   values by rand()%10 as main.cu:236-243, seeded by --seed (the reference
//   seeds with time(NULL)).  --gpus N / --devices: A's rows split over N
//   devices (ias_csr_mul_csr_multi: one host thread + plan per device, B on
//   every device, C concatenated in row order; a device may repeat, which
//   rehearses the split on one GPU); run_time = the slowest device.
#include "ias.h"
#include "report.hpp"

#include <cstring>
#include <string>
#include <vector>

using cli::AlgResult;

int main(int argc, char **argv) {
    const char *file = nullptr, *out_path = nullptr;
    bool aat = false, rand10 = false;
    unsigned seed = 0;
    std::vector<int32_t> devices;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--aat")) aat = true;
        else if (!strcmp(argv[i], "--rand10")) rand10 = true;
        else if (!strcmp(argv[i], "--seed") && i + 1 < argc) seed = (unsigned)atoi(argv[++i]);
        else if (!strcmp(argv[i], "--mtx-out") && i + 1 < argc) out_path = argv[++i];
        else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) {
            devices.clear();
            for (int d = 0, n = atoi(argv[++i]); d < n; ++d) devices.push_back(d);
        } else if (!strcmp(argv[i], "--devices") && i + 1 < argc) {
            devices.clear();
            std::string l = argv[++i];
            for (size_t p = 0; p <= l.size();) {
                size_t q = l.find(',', p);
                if (q == std::string::npos) q = l.size();
                if (q > p) devices.push_back((int32_t)atoi(l.substr(p, q - p).c_str()));
                p = q + 1;
            }
        }
        else if (!file) file = argv[i];
    }
    if (!file) {
        std::printf("please use command like this : ./spgemm-gpu ./sample.mtx\n");
        return 0;
    }
    ias_csr A{}, B{};
    ias_mtx_info info{};
    CLI_TRY("read", ias_mtx_read(file, &A, &info));
    if (rand10) {
        srand(seed);
        for (int64_t i = 0; i < A.nnz; ++i) A.val[i] = rand() % 10;
    }
    // A goes to HBM once; A^T is built there (device transpose replacing
    // mkl_dcsrcsc) and brought back only for the selector's features.
    ias_csr dA{}, dB{};
    CLI_TRY("upload", ias_csr_copy(&A, &dA, IAS_MEMORY_DEVICE, 0));
    if (aat) {
        CLI_TRY("transpose", ias_csr_transpose(&dA, &dB));
        CLI_TRY("copy", ias_csr_copy(&dB, &B, IAS_MEMORY_HOST, 0));
    } else {
        CLI_TRY("copy", ias_csr_copy(&A, &B, IAS_MEMORY_HOST, 0));
        CLI_TRY("upload", ias_csr_copy(&B, &dB, IAS_MEMORY_DEVICE, 0));
    }
    int64_t flops = 0;
    CLI_TRY("flops", ias_flops(&A, &B, &flops));

    // MatNet with the reference's P100 weights over GetInfo1(A), GetInfo1(B)
    // and the two density images (GPU/main.cu:276-460); classes {CUSP,
    // cuSPARSE, NSPARSE}; without weights the hash path (class 1) is assumed.
    const int chosen = cli::matnet_choose(A, B, 18, "p100", 1);
    std::printf("The Chosen One = Algorithm %d\n", chosen + 1);

    ias_opts o;
    ias_opts_default(&o);
    o.output_memory = IAS_MEMORY_DEVICE;
    o.device = 0;
    CLI_TRY("plan", ias_plan_create(&o.plan, 0, nullptr));
    std::vector<AlgResult> r(2);
    const bool multi = devices.size() > 1;
    if (multi) std::printf("row blocks over %zu devices\n", devices.size());
    for (int alg = 0; alg < 2; ++alg) {
        o.order = alg == 0 ? IAS_ORDER_REFERENCE : IAS_ORDER_SORTED;
        ias_csr C{};
        if (multi) {
            ias_opts om = o;
            om.plan = nullptr;
            om.output_memory = IAS_MEMORY_HOST;
            CLI_TRY("spgemm", ias_csr_mul_csr_multi(&dA, &dB, &C, (int32_t)devices.size(), devices.data(), &om,
                                                    nullptr));   // warm-up
            ias_csr_free(&C);
            ias_report rep{};
            CLI_TRY("spgemm", ias_csr_mul_csr_multi(&dA, &dB, &C, (int32_t)devices.size(), devices.data(), &om,
                                                    &rep));
            r[alg].run_ms = rep.ms_total;
            r[alg].mem = ias_sizeof_csr(&C);
            ias_sum_csr(&C, &r[alg].sum);
            if (alg == 0 && out_path) CLI_TRY("write", ias_mtx_write(out_path, &C));
            ias_csr_free(&C);
            continue;
        }
        CLI_TRY("spgemm", ias_csr_mul_csr(&dA, &dB, &C, &o, nullptr));   // warm-up
        ias_csr_free(&C);
        ias_report rep{};
        CLI_TRY("spgemm", ias_csr_mul_csr(&dA, &dB, &C, &o, &rep));
        r[alg].run_ms = rep.ms_total;   // device time (hipEvent), as the reference's cudaEvent timer
        r[alg].mem = ias_sizeof_csr(&C);
        ias_sum_csr(&C, &r[alg].sum);
        if (alg == 0 && out_path) CLI_TRY("write", ias_mtx_write(out_path, &C));
        ias_csr_free(&C);
    }
    ias_plan_destroy(o.plan);
    cli::report(r, (long long)flops, false, false);
    static const char *names[3] = {"CUSP", "cuSPARSE", "NSPARSE"};   // GPU/main.cu:539-544
    if (chosen >= 0 && chosen < 3) std::printf("MatNet predicts Algorithm %s is optimal\n", names[chosen]);
    ias_csr_free(&dA); ias_csr_free(&dB);
    ias_csr_free(&A); ias_csr_free(&B);
    return 0;
}
