/* A plain C99 caller of the drop-in boundary: compiled by gcc against include/pathplanning_amd.h
 * and linked with the HIP library, the way a Rust/C maintainer would consume it.
 * It prints, as one JSON object, the struct layouts the header gives a C compiler and the results
 * of the host-only entry points (no GPU needed), so tests/test_c_consumer.py can check them
 * against the ctypes mirror in pathplanning_amd/_ffi.py and against the C oracle. */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#include "pathplanning_amd.h"

#define OFF(T, f) printf("\"%s.%s\": %zu, ", #T, #f, offsetof(T, f))

int main(void) {
    double xy[2 * 64];
    int n = -1, ndev = -1;
    int rc_circle = pp_create_circle(1.5, -2.0, 3.0, xy, 64, &n);
    int rc_small = pp_create_circle(0.0, 0.0, 3.0, xy, 4, &n);
    int n_small = n;
    pp_create_circle(1.5, -2.0, 3.0, xy, 64, &n);
    int rc_dev = pp_device_count(&ndev);

    printf("{\"abi\": %d, ", pp_abi_version());
    printf("\"sizeof.pp_dubins_config\": %zu, \"sizeof.pp_stats\": %zu, ",
           sizeof(pp_dubins_config), sizeof(pp_stats));
    OFF(pp_dubins_config, sx); OFF(pp_dubins_config, eyaw);
    OFF(pp_dubins_config, turn_radius); OFF(pp_dubins_config, step_size);
    OFF(pp_stats, iterations); OFF(pp_stats, node_evals); OFF(pp_stats, nn_scan_ms);
    OFF(pp_stats, nn_scan_launches); OFF(pp_stats, steer_ms); OFF(pp_stats, steer_launches);
    OFF(pp_stats, walk_points); OFF(pp_stats, batch_steps); OFF(pp_stats, batch_passes);
    OFF(pp_stats, finish_ms); OFF(pp_stats, finish_nodes); OFF(pp_stats, finish_points);
    OFF(pp_stats, reserved_abi3); OFF(pp_stats, samples_evaluated); OFF(pp_stats, samples_blocked);
    OFF(pp_stats, walk_tasks);
    printf("\"rc_circle\": %d, \"rc_small\": %d, \"n_small\": %d, \"n\": %d, ", rc_circle,
           rc_small, n_small, n);
    printf("\"xy\": [");
    for (int i = 0; i < 2 * n; ++i) printf("%s%.17g", i ? ", " : "", xy[i]);
    printf("], \"mod2pi\": %.17g, \"pi_2_pi\": %.17g, ", pp_mod2pi(-7.25), pp_pi_2_pi(4.0));
    printf("\"rng\": \"%llu\", \"gen_range\": %.17g, ", (unsigned long long)pp_rng_u64(42, 7),
           pp_gen_range(42, 7, -3.0, 5.0));
    printf("\"rc_dev\": %d, \"ndev\": %d, \"ok\": %d, \"err\": %d}\n", rc_dev, ndev, PP_OK,
           PP_ERR_CAPACITY);
    return 0;
}
