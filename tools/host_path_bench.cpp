// Host-path latency of the PMPC C ABI without Python: one C2 batch (B = 18) per call.
//   host   : dart_mpc_solve_batch (inputs from host memory, results back in host memory, blocking)
//   dev    : dart_mpc_solve_batch_dev on device-resident inputs + hipStreamSynchronize
//   dev1   : the same with max_iter = 1 (the launch's fixed cost)
//   hipsync: an empty hipStreamSynchronize (no work)
// Build (tools/host_path_bench.sh): hipcc -O2 -I include tools/host_path_bench.cpp -L<pkg>/dart_mpc -ldartmpc
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dart_mpc.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 18, reps = argc > 2 ? atoi(argv[2]) : 2000;
    const char* path = argc > 3 ? argv[3] : "ipopt";
    // C2-like inputs: the first instances of the seeded workload are not needed for latency, a fixed
    // spread of states and targets is (status is checked)
    std::vector<double> x0(6 * B), ref(6 * B), prm(6 * B);
    for (int b = 0; b < B; ++b) {
        const double s = (b % 7) / 7.0 - 0.4, t = (b % 5) / 5.0 - 0.4;
        double xs[6] = {0.18 * s, 0.1 * t, -0.12 * s, 0.05, 0.43, 0.003 * t};
        double rs[6] = {0.15 * t, 0.0, 0.1 * s, 0.0, 0.4, 0.0};
        double ps[6] = {0.05 + 0.05 * (b % 3), 600.0 - 200.0 * (b / 6), 5.0 - 1.5 * (b / 6 > 0), 0.1 + 0.1 * (b >= 6),
                        -0.6, 0.6};
        for (int i = 0; i < 6; ++i) { x0[6 * b + i] = xs[i]; ref[6 * b + i] = rs[i]; prm[6 * b + i] = ps[i]; }
    }
    std::vector<double> u0(2 * B), f(B);
    std::vector<int32_t> st(B), it(B);
    dart_mpc_config cfg;
    dart_mpc_config_default(&cfg);
    cfg.N = 20; cfg.B_max = B; cfg.pmpc_path = (path[0] == 'r');
    dart_mpc_handle* h = nullptr;
    if (dart_mpc_create(&cfg, 0, &h) != 0) { std::printf("create failed\n"); return 1; }
    auto med = [](std::vector<double>& v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };

    std::vector<double> th(reps);
    for (int r = 0; r < 100; ++r) dart_mpc_solve_batch(h, B, x0.data(), ref.data(), prm.data(), nullptr, u0.data(), f.data(), nullptr, st.data(), it.data(), nullptr);
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_us();
        dart_mpc_solve_batch(h, B, x0.data(), ref.data(), prm.data(), nullptr, u0.data(), f.data(), nullptr, st.data(), it.data(), nullptr);
        th[r] = now_us() - t0;
    }
    int nok = 0, itmax = 0;
    for (int b = 0; b < B; ++b) { nok += st[b] == 0; itmax = std::max(itmax, (int)it[b]); }

    double *dx, *dr, *dp, *du, *df; int32_t *ds, *di;
    hipMalloc(&dx, 6 * B * 8); hipMalloc(&dr, 6 * B * 8); hipMalloc(&dp, 6 * B * 8);
    hipMalloc(&du, 2 * B * 8); hipMalloc(&df, B * 8); hipMalloc(&ds, B * 4); hipMalloc(&di, B * 4);
    hipMemcpy(dx, x0.data(), 6 * B * 8, hipMemcpyHostToDevice);
    hipMemcpy(dr, ref.data(), 6 * B * 8, hipMemcpyHostToDevice);
    hipMemcpy(dp, prm.data(), 6 * B * 8, hipMemcpyHostToDevice);
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    std::vector<double> td(reps), t1(reps), ts(reps);
    for (int r = 0; r < 100; ++r) { dart_mpc_solve_batch_dev(h, B, dx, dr, dp, nullptr, du, df, nullptr, ds, di, s); hipStreamSynchronize(s); }
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_us();
        dart_mpc_solve_batch_dev(h, B, dx, dr, dp, nullptr, du, df, nullptr, ds, di, s);
        hipStreamSynchronize(s);
        td[r] = now_us() - t0;
    }
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_us();
        hipStreamSynchronize(s);
        ts[r] = now_us() - t0;
    }
    // back-to-back device launches (the bench's device-resident loop): per-launch wall time
    hipDeviceSynchronize();
    const double tb0 = now_us();
    for (int r = 0; r < reps; ++r) dart_mpc_solve_batch_dev(h, B, dx, dr, dp, nullptr, du, df, nullptr, ds, di, s);
    hipStreamSynchronize(s);
    const double tb = (now_us() - tb0) / reps;
    // the resident server: the same host entry without a kernel launch per call
    std::vector<double> tsv(reps);
    double srv_us = -1.0;
    if (dart_mpc_serve_start(h, B, 5.0) == 0) {
        for (int r = 0; r < 100; ++r) dart_mpc_solve_batch(h, B, x0.data(), ref.data(), prm.data(), nullptr, u0.data(), f.data(), nullptr, st.data(), it.data(), nullptr);
        for (int r = 0; r < reps; ++r) {
            const double t0 = now_us();
            dart_mpc_solve_batch(h, B, x0.data(), ref.data(), prm.data(), nullptr, u0.data(), f.data(), nullptr, st.data(), it.data(), nullptr);
            tsv[r] = now_us() - t0;
        }
        srv_us = med(tsv);
        dart_mpc_serve_stop(h);
    }
    dart_mpc_destroy(h);
    cfg.max_iter = 1;
    dart_mpc_create(&cfg, 0, &h);
    for (int r = 0; r < 100; ++r) { dart_mpc_solve_batch_dev(h, B, dx, dr, dp, nullptr, du, df, nullptr, ds, di, s); hipStreamSynchronize(s); }
    for (int r = 0; r < reps; ++r) {
        const double t0 = now_us();
        dart_mpc_solve_batch_dev(h, B, dx, dr, dp, nullptr, du, df, nullptr, ds, di, s);
        hipStreamSynchronize(s);
        t1[r] = now_us() - t0;
    }
    dart_mpc_destroy(h);
    std::printf("{\"B\": %d, \"path\": \"%s\", \"solved\": %d, \"max_iters\": %d, \"host_us\": %.2f, \"served_us\": %.2f, "
                "\"dev_sync_us\": %.2f, \"dev_back_to_back_us\": %.2f, \"dev_1iter_sync_us\": %.2f, \"empty_sync_us\": %.2f}\n",
                B, path, nok, itmax, med(th), srv_us, med(td), tb, med(t1), med(ts));
    return 0;
}
