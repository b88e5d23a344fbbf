// gossip_protocol_amd/csrc/capi_common.cpp -- status strings, Params parsing, device count.
#include <cstdio>
#include <cstring>

#include "common.hpp"
#include "philox.hpp"

namespace gsp {
namespace {
thread_local std::string g_error;
}
void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_error = buf;
}
const char *get_error() { return g_error.c_str(); }
}  // namespace gsp

extern "C" {

const char *gsp_last_error(void) { return gsp::get_error(); }
int gsp_abi_version(void) { return GSP_ABI_VERSION; }

uint32_t gsp_replay_draw(uint32_t domain, uint64_t seed, uint32_t a, uint32_t b, uint32_t c,
                         uint32_t d) {
    return gsp::draw_u31(domain, seed, a, b, c, d);
}

int gsp_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    GSP_REQUIRE(ctr && key && out, GSP_ERR_INVALID, "gsp_philox4x32_10: NULL argument");
    gsp::philox4x32_10(ctr, key, out);
    return GSP_OK;
}

int gsp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int gsp_params_default(gsp_params *out) {
    GSP_REQUIRE(out, GSP_ERR_INVALID, "gsp_params_default: out is NULL");
    std::memset(out, 0, sizeof *out);
    out->max_nnb = 10;
    out->msg_drop_prob = 0.1;
    out->step_rate = 0.25;           // Params.cpp:30
    out->max_msg_size = 4000;        // Params.cpp:31
    out->en_buff_size = 30000;       // EmulNet.h:12
    out->total_running_time = 700;   // Application.h:27
    out->tremove = 20;               // MP1Node.h:21
    out->id_filter_limit = 10;       // MP1Node.cpp:245
    return GSP_OK;
}

// Same grammar as Params::setparams (Params.cpp:19-26): four fscanf literal prefixes.
int gsp_params_from_conf(const char *path, gsp_params *out) {
    GSP_REQUIRE(path && out, GSP_ERR_INVALID, "gsp_params_from_conf: NULL argument");
    gsp_params_default(out);
    FILE *f = std::fopen(path, "r");
    GSP_REQUIRE(f, GSP_ERR_IO, "gsp_params_from_conf: cannot open %s", path);
    int nnb = 0, single = 0, drop = 0;
    double prob = 0.0;
    int ok = 1;
    ok &= std::fscanf(f, "MAX_NNB: %d", &nnb) == 1;
    ok &= std::fscanf(f, "\nSINGLE_FAILURE: %d", &single) == 1;
    ok &= std::fscanf(f, "\nDROP_MSG: %d", &drop) == 1;
    ok &= std::fscanf(f, "\nMSG_DROP_PROB: %lf", &prob) == 1;
    std::fclose(f);
    GSP_REQUIRE(ok, GSP_ERR_IO, "gsp_params_from_conf: %s is not a MAX_NNB/SINGLE_FAILURE/"
                "DROP_MSG/MSG_DROP_PROB .conf", path);
    out->max_nnb = nnb;
    out->single_failure = single;
    out->drop_msg = drop;
    out->msg_drop_prob = prob;
    return GSP_OK;
}

}  // extern "C"
