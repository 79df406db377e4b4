// alist_to_pchk.cpp -- `alist-to-pchk [-t] alist-file pchk-file`, the same
// command line and file formats as the reference's Neal tool
// (LDPC_dec/ldpc/alist-to-pchk.cpp:36-160), built on the C ABI.
#include <cstdio>
#include <cstring>

#include "../../include/ldpc_amd.h"

int main(int argc, char** argv)
{
    int trans = 0;
    while (argc > 1 && std::strcmp(argv[1], "-t") == 0) {
        trans = 1;
        argc--;
        argv++;
    }
    if (argc != 3) {
        std::fprintf(stderr, "Usage: alist-to-pchk [ -t ] alist-file pchk-file\n");
        return 1;
    }
    int err = 0;
    ldpc_graph* g = ldpc_graph_load_alist(argv[1], trans, &err);
    if (!g) {
        std::fprintf(stderr, "%s\n", ldpc_last_error());
        return 1;
    }
    if (ldpc_graph_save_pchk(g, argv[2]) != LDPC_OK) {
        std::fprintf(stderr, "%s\n", ldpc_last_error());
        ldpc_graph_free(g);
        return 1;
    }
    ldpc_graph_free(g);
    return 0;
}
