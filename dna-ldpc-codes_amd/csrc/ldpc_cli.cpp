// ldpc_cli.cpp -- file-compatible replacement of the reference's ldpc.exe for
// the DNA pipeline's call (def_func.py:47-51):
//
//   ldpc <bSystematic> <decoder_type> <channel_type> <seed> <max_iter> <frame_num>
//        [<target_frame_err> if frame_num == 0] <codeword_base> <soft_base> <pchk_base>
//        <EbNo | eps (BEC) | p (BSC)> <punct> <short> <target> [punct/short/target args]
//
// Argument parsing follows SetUp (DNA_main.cpp:300-505) for this subset;
// decoder_type 0 = BP (dec.cpp:583), 20/21/22 = float min-sum (dec.cpp:1216,
// with g_precision = 0, DNA_main.cpp:1293-1296, 1588-1594), 1/2/3 = Gallager
// A/B1/B2 (dec.cpp:699).  Inputs: <codeword>.txt
// (N ints, error statistics only), <soft>.txt (N LLRs, LR = exp(LLR),
// DNA_main.cpp:1319-1345), <pchk>.pchk.  Outputs: dec_<codeword>.txt ("%d "
// per bit, DNA_main.cpp:916-927), result_(<soft>.txt)_<pchk>.pchk_... .txt
// (Print_All_Result, DNA_main.cpp:965-1123), stdout summary (Set_Code :551-556,
// Print_One_Result :1170-1182).  The decode itself runs on the GPU through the
// C ABI; there is no CPU decode path.
//
// Puncturing / shortening (SetUp :333-478, Set_Code :565-605, LDPC_Channel
// :1375-1418): the argv and the side files (<pchk>.txt with the SC-code
// multiplicities for types 2-4, <pchk>_punct.txt for type 5) are read as the
// reference reads them; the code rate (and g_std_dev) and the result-file
// lines follow.  On the AWGN / BSC channels the reference edits only the
// received LR: punctured bits get LR = 1 (types 1, 2), shortened bits LR =
// exp(30) (type 1, AWGN).  BP decodes from that LR, so this build passes LLR 0
// / 30.0, whose host exp is the same LR bit for bit; min-sum and Gallager
// read the unedited LLR / hard input, as in the reference.  Types 3-5 and BEC
// erasure marks only change the hard input of the BEC decoders, which are
// out of scope.  Indices outside the code, and shortening type 2 with an
// SC-code length (undefined behaviour in the reference: LR[-1]), exit 1.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "../../include/ldpc_amd.h"
#include "cli_io.hpp"

// the loaded graph, freed at exit on every path (die() exits directly)
static ldpc_graph* g_graph = nullptr;
static void free_graph() { if (g_graph) ldpc_graph_free(g_graph); g_graph = nullptr; }

static void die(const char* msg)
{
    std::fprintf(stderr, "%s\n", msg);
    std::exit(1);
}

// bounds on argv-sized work that the reference leaves unchecked
constexpr long long kMaxSideInts = 1LL << 24;   // entries of an SC-code side file
constexpr long long kMaxFrames = 1LL << 40;     // frame counters stay far from int64 overflow

int main(int argc, char** argv)
{
    // ---- SetUp (DNA_main.cpp:300-331, 494-502) ----
    int pos = 1;
    auto arg = [&](void) -> const char* {
        if (pos >= argc) { std::fprintf(stderr, "\n\nargc error!\n\n"); std::exit(1); }
        return argv[pos++];
    };
    const int bSystematic = std::atoi(arg());
    const int decoder_type = std::atoi(arg());
    const int channel_type = std::atoi(arg());
    const int seed = std::atoi(arg());
    const int max_iter = std::atoi(arg());
    const long frame_num = std::atol(arg());
    int target_frame_err = 0;
    if (frame_num == 0) target_frame_err = std::atoi(arg());
    const std::string cw_base = arg();
    const std::string soft_base = arg();
    const std::string pchk_base = arg();
    double EbNo = 0, eps = 0, p = 0;
    if (channel_type == 2) eps = std::atof(arg());
    else if (channel_type == 1) p = std::atof(arg());
    else EbNo = std::atof(arg());
    const int punct = std::atoi(arg());
    const int shortening = std::atoi(arg());
    const int targeting = std::atoi(arg());
    int p_start = 0, p_end = 0, p_start1 = 0, p_end1 = 0, p_start2 = 0, p_end2 = 0;
    int s_start = 0, s_end = 0, s_etha = 0, s_num = 0, sc_w = 0, sc_L = 0;
    std::vector<int> sc_M;  // g_SC_CODE_M (types 2-4)
    int target_VN[2] = {0, 0};
    if (punct > 0 && punct != 5) { p_start = std::atoi(arg()); p_end = std::atoi(arg()); }
    if (shortening == 1) { s_start = std::atoi(arg()); s_end = std::atoi(arg()); }
    if (shortening == 2) { s_etha = std::atoi(arg()); s_num = std::atoi(arg()); }
    if (targeting) { target_VN[0] = std::atoi(arg()); target_VN[1] = std::atoi(arg()); }
    auto read_ints = [&](const std::string& path, long long n, std::vector<int>& out) {
        // a short file leaves the calloc'd zeros, as fscanf does
        std::string msg;
        if (n > kMaxSideInts) die("ldpc: SC-code side file length out of range");
        if (!ldpc_cli::read_int_file(path, (size_t)n, /*allow_short=*/true, out, &msg)) die(("ldpc: " + msg).c_str());
    };
    if (punct >= 2 && punct <= 4) {
        // SetUp :355-431: [start1 end1 (type 4)] w L, <pchk>.txt holds D = L + w - 1
        // multiplicities (and, for type 2, D more that only the SC decoders use)
        if (punct == 4) { p_start1 = std::atoi(arg()); p_end1 = std::atoi(arg()); }
        sc_w = std::atoi(arg());
        sc_L = std::atoi(arg());
        const long long D = (long long)sc_L + sc_w - 1;
        if (sc_L < 0 || D < 0 || (D < sc_L)) die("ldpc: SC-code w / L out of range");
        read_ints(pchk_base + ".txt", D, sc_M);
        if (punct >= 3) { p_start2 = std::atoi(arg()); p_end2 = std::atoi(arg()); }
    }
    if (punct == 5 && sc_L > 0) {  // SetUp :468-478 reads g_SC_CODE_L entries (0 outside SC runs)
        std::vector<int> unused;
        read_ints(pchk_base + "_punct.txt", sc_L, unused);
    }
    if (argc != pos) { std::fprintf(stderr, "\n\nargc error!\n\n"); return 1; }
    int algo;
    // LDPC_Decode DNA_main.cpp:1565-1594.  The DNA build never sets
    // g_precision (0), so 20/21/22 all run the float min-sum
    // Run_MSA_Decoder_INF; Gallager 1/2/3 decode the hard decision of the
    // soft input (the reference's DNA build leaves g_recv_codeword_hard unset).
    if (decoder_type == 0) algo = LDPC_ALGO_BP;
    else if (decoder_type == 20 || decoder_type == 21 || decoder_type == 22) algo = LDPC_ALGO_MSA;
    else if (decoder_type == 1) algo = LDPC_ALGO_GALLAGER_A;
    else if (decoder_type == 2) algo = LDPC_ALGO_GALLAGER_B1;
    else if (decoder_type == 3) algo = LDPC_ALGO_GALLAGER_B2;
    else die("ldpc: decoder_type must be 0 (BP), 1/2/3 (Gallager A/B1/B2) or 20/21/22 (min-sum)");
    (void)eps; (void)p;

    const std::string file_cw = cw_base + ".txt", file_soft = soft_base + ".txt", file_pchk = pchk_base + ".pchk";

    // ---- Set_Code (DNA_main.cpp:544-609) ----
    int err = 0;
    ldpc_graph* g = ldpc_graph_load(file_pchk.c_str(), &err);
    g_graph = g;
    std::atexit(free_graph);
    if (!g) { std::fprintf(stderr, "%s\n", ldpc_last_error()); return 1; }
    int32_t M, N, dv, rdv, dc, rdc;
    int64_t E;
    ldpc_graph_info(g, &M, &N, &E, &dv, &rdv, &dc, &rdc);
    const int K = N - M;
    std::printf("\n");
    std::printf("g_CODE_N : %d\n", N);
    std::printf("g_CODE_K : %d\n", K);
    std::printf("g_CODE_M : %d\n", M);
    std::printf("\n");
    if (!targeting) { target_VN[0] = 1; target_VN[1] = N; }
    // LDPC_BIT_Check indexes codeword[target_VN[0]-1 .. target_VN[1]-1] unchecked (DNA_main.cpp:1675-1706)
    if (target_VN[0] < 1 || target_VN[1] > N || target_VN[0] > target_VN[1]) die("ldpc: target_VN range outside the code");
    double rate;  // Set_Code :565-605 (g_rand_type = RAND_SEED, g_save_type = 0 in this build)
    if (punct == 1) {
        const double np = (double)p_end - p_start + 1;
        rate = 1.0 - ((double)M - np) / ((double)N - np);
    } else if (punct >= 2 && punct <= 4) {
        long long np = ((long long)p_end - p_start + 1) * sc_L;
        if (punct >= 3) np += (long long)p_end2 - p_start2 + 1;
        if (punct == 4) np += ((long long)p_end1 - p_start1 + 1) * (sc_w - 1);
        rate = 1.0 - (double)(M - np) / (double)(N - np);
    } else if (shortening == 1) {
        rate = 1.0 - (double)M / ((double)N - ((double)s_end - s_start + 1));
    } else if (shortening == 2) {
        if (s_etha == 0) die("ldpc: shortening type 2 needs a nonzero period");
        const int ns = (int)(s_num * std::floor((double)sc_L / (double)s_etha));
        rate = 1.0 - (double)M / (double)(N - ns);
    } else {
        rate = 1.0 - (double)M / (double)N;
    }
    const double std_dev = 1 / std::sqrt(2 * rate * std::pow(10.0, EbNo * 0.1));  // getStd_dev channel.cpp:9-16

    time_t t_start, t_end;
    std::time(&t_start);

    // ---- LDPC_Encode: read codeword + LLR (DNA_main.cpp:1319-1345) ----
    // cli_io.hpp: a missing file, fewer than N values or a non-numeric token
    // exit 1 (the reference runs on with stale or zero values)
    std::vector<int> codeword;
    std::vector<double> llr;
    std::string io_msg;
    if (!ldpc_cli::read_int_file(file_cw, (size_t)N, /*allow_short=*/false, codeword, &io_msg) ||
        !ldpc_cli::read_double_file(file_soft, (size_t)N, llr, &io_msg))
        die(("ldpc: " + io_msg).c_str());

    // ---- LDPC_Channel raw error count (DNA_main.cpp:1711-1748) ----
    const int len_raw = bSystematic ? K : N;
    long long raw = 0;
    for (int i = 0; i < len_raw; i++) {
        int temp;
        if (channel_type == 0) temp = llr[(size_t)i] >= 0 ? 0 : 1;
        else if (channel_type == 2) { continue; }  // hard input never set -> no erasure marks
        else temp = 0;                             // BSC: hard input never set (channel sims disabled)
        if (codeword[(size_t)i] != temp) raw++;
    }

    // ---- LDPC_Channel's LR edits (:1375-1441), seen by BP only ----
    std::vector<double> llr_bp(llr);
    auto set_lr = [&](long idx, double v) {
        if (idx < 0 || idx >= N) die("ldpc: punctured / shortened bit outside the code");
        llr_bp[(size_t)idx] = v;  // LR = exp(v): exp(30.0), exp(0) = 1
    };
    if (shortening == 1 && channel_type == 0)
        for (int i = s_start; i <= s_end; i++) set_lr(i - 1, 30.0);
    if (shortening == 2 && channel_type == 0 && sc_L > 0)
        die("ldpc: shortening type 2 with an SC-code length indexes LR[-1] in the reference (undefined)");
    if (channel_type == 0 || channel_type == 1) {
        if (punct == 1) {
            for (int i = p_start; i <= p_end; i++) set_lr(i - 1, 0.0);
        } else if (punct == 2) {
            long idx = 0;
            for (int j = 0; j < sc_L; j++) {
                for (int i = p_start; i <= p_end; i++) set_lr(idx + i - 1, 0.0);
                idx += sc_M[(size_t)j];
            }
        }
    }

    // ---- LDPC_Decode on the GPU ----
    std::vector<uint8_t> hard((size_t)N);
    int32_t iters = 0;
    uint8_t valid = 0;
    ldpc_opts o{};
    o.exp_on_host = 1;
    const double* in = algo == LDPC_ALGO_BP ? llr_bp.data() : llr.data();
    if (ldpc_decode(g, in, 1, max_iter, algo, hard.data(), nullptr, &iters, &valid, &o) != LDPC_OK) {
        std::fprintf(stderr, "ldpc: decode failed: %s\n", ldpc_last_error());
        return 1;
    }

    // ---- LDPC_BIT_Check (DNA_main.cpp:1675-1706) ----
    long long bit_err = 0;
    if (bSystematic) {
        for (int i = 0; i < K; i++) bit_err += codeword[(size_t)i] != hard[(size_t)i];
    } else {
        for (int i = target_VN[0] - 1; i < target_VN[1]; i++) bit_err += codeword[(size_t)i] != hard[(size_t)i];
    }

    // ---- frame loop bookkeeping (Check_End :756-795; Run_Simulation :800-912) ----
    // Every frame re-reads the same files and decodes identically, so the
    // counters scale with the number of frames.
    long long frames;
    if (frame_num == 0) {
        if (target_frame_err <= 0) frames = 0;
        else if (bit_err > 0) frames = target_frame_err;
        else die("ldpc: frame_num 0 with an error-free decode never reaches the target frame-error count");
    } else {
        frames = frame_num;
    }
    if (frames > kMaxFrames) die("ldpc: frame_num out of range");
    long long frame_i[3] = {frames, frames, 0};
    long long bit_errs[3] = {raw * frames, bit_err * frames, bit_err * frames};
    long long frame_errs[3] = {raw > 0 ? frames : 0, bit_err > 0 ? frames : 0, bit_err > 0 ? frames : 0};

    const std::string file_dec = "dec_" + cw_base + ".txt";
    std::printf("%s", file_dec.c_str());
    FILE* fd = std::fopen(file_dec.c_str(), "w");
    if (!fd) die("ldpc: cannot write the decoded-word file");
    for (int i = 0; i < N; i++) std::fprintf(fd, "%d ", frames > 0 ? (int)hard[(size_t)i] : 0);
    std::fclose(fd);
    std::time(&t_end);

    // ---- Print_One_Result (DNA_main.cpp:1170-1182) ----
    std::printf("\n");
    if (channel_type == 2)
        std::printf("[%d]  code : (%d,%d)\trate : %.3f\tEps : %.2f \n", 0, N, K, rate, eps);
    else
        std::printf("[%d]  code : (%d,%d)\trate : %.3f\tEb/No : %.2f dB\n", 0, N, K, rate, EbNo);
    std::printf("[%d]  frame_num              : %lld\n", 0, frame_i[0]);
    std::printf("[%d]  bit_err                : %lld\n", 0, bit_errs[2]);
    std::printf("[%d]  frame_err              : %lld\n", 0, frame_errs[2]);
    std::printf("[%d]  without coding (bit)   : %lld\n", 0, bit_errs[0]);
    std::printf("[%d]  without coding (frame) : %lld\n\n", 0, frame_errs[0]);

    // ---- Print_All_Result (DNA_main.cpp:965-1123) ----
    const int len = bSystematic ? K : (target_VN[1] - target_VN[0] + 1);
    const double denom = (double)len * (double)frame_i[0];
    double BER[3];
    for (int i = 0; i < 3; i++) BER[i] = (double)bit_errs[i] / denom;
    const std::string file_soft_txt = soft_base + ".txt";
    char name[4096];
    if (channel_type == 2)
        std::snprintf(name, sizeof name, "result_(%s)_%s_%d_%.3f_%d_%d_%d.txt", file_soft_txt.c_str(), file_pchk.c_str(),
                      decoder_type, eps, 0, max_iter, seed);
    else if (channel_type == 1)
        std::snprintf(name, sizeof name, "result_(%s)_%s_%d_%.4f_%d_%d_%d.txt", file_soft_txt.c_str(), file_pchk.c_str(),
                      decoder_type, p, 0, max_iter, seed);
    else
        std::snprintf(name, sizeof name, "result_(%s)_%s_%d_%.3fdB_%d_%d_%d.txt", file_soft_txt.c_str(),
                      file_pchk.c_str(), decoder_type, EbNo, 0, max_iter, seed);
    FILE* fr = std::fopen(name, "w");
    if (!fr) die("ldpc: cannot write the result file");
    std::fprintf(fr, "code N        : %d\n", N);
    std::fprintf(fr, "code K        : %d\n", K);
    std::fprintf(fr, "code M        : %d\n", M);
    std::fprintf(fr, "code rate     : %.3f\n", rate);
    if (channel_type == 2) {
        std::fprintf(fr, "Eps\t\t: %.3f \n", eps);
    } else {
        std::fprintf(fr, "Eb/No         : %.2f dB\n", EbNo);
        std::fprintf(fr, "g_std_dev     : %.2f\n", std_dev);
    }
    std::fprintf(fr, "max iteration : %d\n", max_iter);
    std::fprintf(fr, "dv            : %d\n", dv);
    std::fprintf(fr, "bRegular_dv   : %d\n", rdv);
    std::fprintf(fr, "dc            : %d\n", dc);
    std::fprintf(fr, "bRegular_dc   : %d\n", rdc);
    if (targeting) std::fprintf(fr, "target_VN:%d~%d \n\n", target_VN[0], target_VN[1]);
    if (punct) std::fprintf(fr, "[Type: %d] Punctuation_VN:%d~%d \n\n", punct, p_start, p_end);
    if (shortening == 1) std::fprintf(fr, "[Type: %d] Shortening_VN:%d~%d \n\n", shortening, s_start, s_end);
    std::fprintf(fr, "=============================================\n");
    std::fprintf(fr, "                 result\n");
    std::fprintf(fr, "=============================================\n");
    double d = std::difftime(t_end, t_start);
    const int hh = (int)(d / 3600);
    d -= hh * 3600;
    const int mm = (int)(d / 60);
    d -= mm * 60;
    const int ss = (int)d;
    std::fprintf(fr, "start time      : %s", std::ctime(&t_start));
    std::fprintf(fr, "end time        : %s", std::ctime(&t_end));
    std::fprintf(fr, "simulation time : %d hours %d mins %d secs\n\n", hh, mm, ss);
    std::fprintf(fr, "# of processes         : %d\n", 1);
    std::fprintf(fr, "initial seed value     : %d\n\n", seed);
    for (int i = 0; i < 2; i++) std::fprintf(fr, "# of Frame[%2d]          :%lld\n", i, frame_i[i]);
    std::fprintf(fr, "\n");
    for (int i = 0; i < 2; i++) std::fprintf(fr, "# of Bit Errors[%2d]     : %lld\n", i, bit_errs[i]);
    std::fprintf(fr, "\n");
    for (int i = 0; i < 2; i++) std::fprintf(fr, "BER[%2d]                 : %.5e\n", i, BER[i]);
    std::fprintf(fr, "\n");
    std::fclose(fr);
    free_graph();
    (void)iters; (void)valid;
    return 0;
}
