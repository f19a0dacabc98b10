// Host-only AddressSanitizer / UBSan run of the symbolic planner (python-mpc_amd/csrc/plan.cpp):
// reads CSC sparsity patterns written by tools/asan/run.sh (one file per layout: n m nnzP nnzA,
// then Pp, Pi, Ap, Ai as int32) and builds the plan with and without eliminated columns.
// Test infrastructure only; built with g++ -fsanitize=address,undefined.
#include <cstdio>
#include <vector>

#include "plan.h"

int main(int argc, char** argv) {
    int bad = 0;
    for (int a = 1; a < argc; ++a) {
        FILE* f = std::fopen(argv[a], "rb");
        if (!f) { std::fprintf(stderr, "cannot open %s\n", argv[a]); return 2; }
        int hdr[4];
        if (std::fread(hdr, sizeof(int), 4, f) != 4) return 2;
        const int n = hdr[0], m = hdr[1], nnzP = hdr[2], nnzA = hdr[3];
        std::vector<int> Pp(n + 1), Pi(nnzP), Ap(n + 1), Ai(nnzA);
        bool ok = std::fread(Pp.data(), sizeof(int), n + 1, f) == (size_t)(n + 1) &&
                  std::fread(Pi.data(), sizeof(int), nnzP, f) == (size_t)nnzP &&
                  std::fread(Ap.data(), sizeof(int), n + 1, f) == (size_t)(n + 1) &&
                  std::fread(Ai.data(), sizeof(int), nnzA, f) == (size_t)nnzA;
        std::fclose(f);
        if (!ok) return 2;
        for (int el = 0; el < 2; ++el) {
            mpcqp::Plan pl;
            const std::string err = mpcqp::build_plan(n, m, Pp.data(), Pi.data(), Ap.data(), Ai.data(), pl, el != 0);
            std::printf("%s eliminate=%d: %s nb=%d npad=%d ne=%d amax=%d gather_k=%d\n", argv[a], el,
                        err.empty() ? "ok" : err.c_str(), pl.nb, pl.npad, pl.ne, pl.amax, pl.gather_k);
            // an unsupported pattern must be refused with a message, never planned partially
            if (!err.empty() && pl.nb != 0) bad = 1;
        }
    }
    return bad;
}
