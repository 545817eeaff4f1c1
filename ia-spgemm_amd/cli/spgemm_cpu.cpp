// spgemm-cpu — drop-in for IA-SPGEMM-CPU_release/main.cpp (the `spgemm-cpu`
// program).  Same argv shape and report; the five algorithms are
//   1 MKL mkl_sparse_sp2m on the host cores (the reference's baseline),
//   2 CSR, 3 DIA, 4 ELL, 5 COO on the MI355X through libias.so.
// Usage: spgemm-cpu A.mtx [B.mtx] [testing_mode 0|1] [--no-warmup]
//                   [--time-scale S]   (timeout harness, default 20; 0 = off)
//   B defaults to A (C = A*A, the README's intent; the reference's own
//   argv[3] read before the argc check is undefined behaviour, main.cpp:99).
// "The Chosen One" comes from MatNet run natively (libias: the reference's
// Intel weights, exported from NetWeights/Intel_weights.h5) instead of
// embedded CPython/Keras.  Other differences, documented in INTEGRATION.md: the
// 20x-MKL timeout is a verdict on the measured time (no cancellation); trans_time prints the measured device-side
// CSRtoX of A (the reference prints uninitialised slots).
#include "ias.h"
#include "report.hpp"

#include <sys/stat.h>

#include <cstring>

using cli::AlgResult;

static bool file_exists(const char *p) {
    struct stat st;
    return stat(p, &st) == 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::printf("please use command like this : ./spgemm-cpu A.mtx [B.mtx] [testing_mode]\n");
        return 0;
    }
    bool warm = true;
    double time_scale = 20.0;   // main.cpp:510
    std::vector<const char *> pos;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--no-warmup")) warm = false;
        else if (!strcmp(argv[i], "--time-scale") && i + 1 < argc) time_scale = atof(argv[++i]);
        else pos.push_back(argv[i]);
    }
    const char *fa = pos[0];
    const char *fb = fa;
    int testing_mode = 0;
    if (pos.size() == 2) {
        if (!file_exists(pos[1]) && sscanf(pos[1], "%d", &testing_mode) == 1) fb = fa;
        else fb = pos[1];
    } else if (pos.size() >= 3) {
        fb = pos[1];
        sscanf(pos[2], "%d", &testing_mode);
    }
    std::printf("-------------- %s, %s --------------\n", fa, fb);
    ias_csr A{}, B{};
    ias_mtx_info ia{}, ib{};
    CLI_TRY("read", ias_mtx_read_pair(fa, fb, &A, &B, &ia, &ib));
    std::printf("Weight Matrix (A): %lldx%lld: symmetric = %s\n", (long long)ia.rows, (long long)ia.cols,
                ia.is_symmetric ? "true" : "false");
    std::printf("Activation Matrix (B): %lldx%lld: symmetric = %s\n", (long long)ib.rows,
                (long long)ib.cols, ib.is_symmetric ? "true" : "false");
    std::printf(ia.is_symmetric ? "Mat A symmetric \n" : "Mat A non-symmetric \n");
    std::printf(ib.is_symmetric ? "Mat B symmetric\n" : "Mat B non-symmetric\n");
    if (testing_mode) {
        std::printf("A_csr:\n");
        cli::print_csr(A);
        std::printf("\nB_csr:\n");
        cli::print_csr(B);
        std::printf("\n");
    }
    std::printf("------------------------------------------\n");

    // ---- formats + selector (MatNet over GetInfo1/2/3 features and density images).
    // A and B go to HBM once; CSRtoDIA/ELL/COO run on the device (convert_dev.hip)
    // and trans_time is that conversion of A, as the reference times its
    // host-side CSRtoX of A (main.cpp:884-930).
    ias_csr dA{}, dB{};
    CLI_TRY("upload", ias_csr_copy(&A, &dA, IAS_MEMORY_DEVICE, 0));
    CLI_TRY("upload", ias_csr_copy(&B, &dB, IAS_MEMORY_DEVICE, 0));
    if (warm) {   // first launches load the conversion kernels' code object
        ias_coo w{};
        if (ias_csr_to_coo(&dA, &w, 0.0) == IAS_SUCCESS) ias_coo_free(&w);
    }
    ias_dia Ad{}, Bd{};
    ias_ell Ae{}, Be{};
    ias_coo Ac{}, Bc{};
    double t0 = cli::now_ms();
    ias_status sd = ias_csr_to_dia(&dA, &Ad, 50.0);
    const double dia_trans = cli::now_ms() - t0;
    ias_status sd2 = ias_csr_to_dia(&dB, &Bd, 50.0);
    t0 = cli::now_ms();
    ias_status se = ias_csr_to_ell(&dA, &Ae, 50.0);
    const double ell_trans = cli::now_ms() - t0;
    ias_status se2 = ias_csr_to_ell(&dB, &Be, 50.0);
    t0 = cli::now_ms();
    ias_status sc = ias_csr_to_coo(&dA, &Ac, 50.0);
    const double coo_trans = cli::now_ms() - t0;
    ias_status sc2 = ias_csr_to_coo(&dB, &Bc, 50.0);
    const bool dia_ok = sd == IAS_SUCCESS && sd2 == IAS_SUCCESS;
    const bool ell_ok = se == IAS_SUCCESS && se2 == IAS_SUCCESS;
    const bool coo_ok = ell_ok && sc == IAS_SUCCESS && sc2 == IAS_SUCCESS;   // main.cpp:917 gates COO on ELL
    const double dia_fill = Ad.num_diagonals ? (double)A.nnz / ((double)Ad.num_diagonals * A.rows) : 0.0;
    const double ell_fill = Ae.max_nnz_per_row ? (double)A.nnz / ((double)Ae.max_nnz_per_row * A.rows) : 0.0;
    const int chosen = cli::matnet_choose(A, B, 26, "intel",
                                          cli::select_format(dia_ok, dia_fill, ell_ok, ell_fill));
    std::printf("The Chosen One = Algorithm %d\n", chosen + 1);

    std::vector<AlgResult> r(5);
    int64_t flops = 0;
    CLI_TRY("flops", ias_flops(&A, &B, &flops));

    // ---- 1 MKL (host)
    {
        ias_csr C{};
        double ms = 0;
        ias_status s = ias_mkl_sp2m(&A, &B, &C, 0, &ms);
        if (s == IAS_SUCCESS) {
            r[0].run_ms = ms;
            r[0].mem = ias_sizeof_csr(&C);
            ias_sum_csr(&C, &r[0].sum);
            if (testing_mode) cli::print_csr(C);
            ias_csr_free(&C);
        } else {
            std::printf("MKL unavailable: %s\n", ias_last_error());
        }
        std::printf("DONE MKL\n");
    }

    ias_opts o;
    ias_opts_default(&o);
    o.output_memory = IAS_MEMORY_DEVICE;
    o.device = 0;
    CLI_TRY("plan", ias_plan_create(&o.plan, 0, nullptr));

    // ---- 2 CSR (device-resident operands, as the reference uploads before timing)
    {
        ias_csr C{};
        if (warm) {
            CLI_TRY("csr", ias_csr_mul_csr(&dA, &dB, &C, &o, nullptr));
            ias_csr_free(&C);
        }
        const double t = cli::now_ms();
        CLI_TRY("csr", ias_csr_mul_csr(&dA, &dB, &C, &o, nullptr));
        r[1].run_ms = cli::now_ms() - t;
        r[1].mem = ias_sizeof_csr(&C);
        ias_sum_csr(&C, &r[1].sum);
        ias_csr_free(&C);
        std::printf("DONE CSR\n");
    }
    // ---- 3 DIA
    if (dia_ok) {
        ias_dia C{};
        if (warm) {
            CLI_TRY("dia", ias_dia_mul_dia(&Ad, &Bd, &C, &o, nullptr));
            ias_dia_free(&C);
        }
        const double t = cli::now_ms();
        CLI_TRY("dia", ias_dia_mul_dia(&Ad, &Bd, &C, &o, nullptr));
        r[2].run_ms = cli::now_ms() - t;
        r[2].trans_ms = dia_trans;
        r[2].mem = ias_sizeof_dia(&C);
        ias_sum_dia(&C, &r[2].sum);
        ias_dia_free(&C);
    }
    std::printf("DONE DIA\n");
    // ---- 4 ELL
    if (ell_ok) {
        ias_ell C{};
        if (warm) {
            CLI_TRY("ell", ias_ell_mul_ell(&Ae, &Be, &C, &o, nullptr));
            ias_ell_free(&C);
        }
        const double t = cli::now_ms();
        CLI_TRY("ell", ias_ell_mul_ell(&Ae, &Be, &C, &o, nullptr));
        r[3].run_ms = cli::now_ms() - t;
        r[3].trans_ms = ell_trans;
        r[3].mem = ias_sizeof_ell(&C);
        ias_sum_ell(&C, &r[3].sum);
        ias_ell_free(&C);
    }
    std::printf("DONE ELL\n");
    // ---- 5 COO
    if (coo_ok) {
        ias_coo C{};
        if (warm) {
            CLI_TRY("coo", ias_coo_mul_coo(&Ac, &Bc, &C, &o, nullptr));
            ias_coo_free(&C);
        }
        const double t = cli::now_ms();
        CLI_TRY("coo", ias_coo_mul_coo(&Ac, &Bc, &C, &o, nullptr));
        r[4].run_ms = cli::now_ms() - t;
        r[4].trans_ms = coo_trans;
        r[4].mem = ias_sizeof_coo(&C);
        ias_sum_coo(&C, &r[4].sum);
        ias_coo_free(&C);
    }
    std::printf("DONE COO\n");
    ias_plan_destroy(o.plan);
    ias_dia_free(&Ad); ias_dia_free(&Bd);
    ias_ell_free(&Ae); ias_ell_free(&Be);
    ias_coo_free(&Ac); ias_coo_free(&Bc);
    ias_csr_free(&dA); ias_csr_free(&dB);

    for (int i = 1; i < 5; ++i) cli::over_deadline(r[i], r[0].run_ms, time_scale);
    const int best = cli::report(r, (long long)flops, true, true);
    double best_sp = best >= 0 ? (r[best].run_ms == 0 ? 0 : r[0].run_ms / r[best].run_ms) : 0.0;
    std::printf("MAX SPEED IS %lf for ALGORITHM %d\n", best_sp, best + 1);
    std::printf("------------------------------\n");
    if (chosen == best) std::printf("Congratulate! MatNet Correct Prediction.\n");
    else std::printf("Unfortunately! MatNet Incorrect Prediction.\n");
    std::printf("------------------------------\n");

    ias_csr_free(&A); ias_csr_free(&B);
    return 0;
}
