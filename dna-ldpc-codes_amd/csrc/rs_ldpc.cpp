// rs_ldpc.cpp -- `rs-ldpc s rho gamma out_filename H_pri`: the command line,
// alist output file and stdout modes of the reference's RS_LDPC
// (RS LDPC encode/RS_LDPC/RS_LDPC.c:221-527), built on the C ABI.
//   H_pri 0: N, M, the generator polynomial and the coset table
//   H_pri 1: the dense H, one row per line
//   else   : "M N"
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/ldpc_amd.h"

int main(int argc, char** argv)
{
    if (argc != 6) {
        std::printf("Incorrect input arguments. Check again.\n");
        std::printf("[Usage] ./RS_LDPC [s] [rho] [gamma] [out_filename]\n");
        return 0;  // RS_LDPC.c:254-259 exits 0
    }
    const int s = std::atoi(argv[1]), rho = std::atoi(argv[2]), gamma = std::atoi(argv[3]);
    const int H_pri = std::atoi(argv[5]);
    if (s < 2 || s > 10 || rho < 3) {
        std::fprintf(stderr, "rs-ldpc: unsupported parameters\n");
        return 1;
    }
    const int q = 1 << s;
    std::vector<int32_t> gp((size_t)rho - 1), coset((size_t)q * q);
    int err = 0;
    ldpc_graph* g = ldpc_graph_rs_ldpc(s, rho, gamma, gp.data(), coset.data(), &err);
    if (!g) {
        std::fprintf(stderr, "%s\n", ldpc_last_error());
        return 1;
    }
    if (ldpc_graph_save_alist(g, argv[4]) != LDPC_OK) {
        std::fprintf(stderr, "%s\n", ldpc_last_error());
        ldpc_graph_free(g);
        return 1;
    }
    int32_t M, N, dv, rdv, dc, rdc;
    int64_t E;
    ldpc_graph_info(g, &M, &N, &E, &dv, &rdv, &dc, &rdc);
    if (H_pri == 0) {
        std::printf("N = %d\nM = %d\n", N, M);
        std::printf("Generator polynomial\n");
        for (int i = 0; i < rho - 1; i++) std::printf("%d ", gp[(size_t)i]);
        std::printf("\n");
        std::printf("Coset\n");
        for (int i = 0; i < q * q; i++) std::printf("%d ", coset[(size_t)i]);
        std::printf("\n");
    } else if (H_pri == 1) {
        std::vector<int32_t> rp((size_t)M + 1), ci((size_t)E), cp((size_t)N + 1), ce((size_t)E);
        ldpc_graph_edges(g, rp.data(), ci.data(), cp.data(), ce.data());
        std::vector<char> row((size_t)N);
        for (int i = 0; i < M; i++) {
            std::fill(row.begin(), row.end(), 0);
            for (int32_t e = rp[(size_t)i]; e < rp[(size_t)i + 1]; e++) row[(size_t)ci[(size_t)e]] = 1;
            for (int j = 0; j < N; j++) std::fputs(row[(size_t)j] ? "1 " : "0 ", stdout);
            std::printf("\n");
        }
    } else {
        std::printf("%d %d", M, N);
    }
    ldpc_graph_free(g);
    return 0;
}
