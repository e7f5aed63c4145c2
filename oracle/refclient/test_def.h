// oracle/refclient/test_def.h -- OUR loopback configuration for the reference's
// unchanged echo client, tests/new-ws-echo/test_ws_client.cpp (compiled from
// its place under /root/reference by oracle/Makefile `refclient`, fed to g++
// on stdin so that this header -- not the reference's test_def.h with its
// hard-coded LAN address and TLS -- is the one its `#include "test_def.h"`
// finds). Same names and meaning as tests/new-ws-echo/test_def.h:1-40; the
// values are plain ws:// on 127.0.0.1 with 4 KiB messages (BASELINE config 1).
// TEST INFRASTRUCTURE: the GPU test tests/test_gpu_dropin.py runs the built
// client against the GPU-hooked drop-in server so the client's own HashArr
// check (test_ws_client.cpp:260-277) sees bytes the MI355X unmasked.
// With FWS_REFSERVER_GPU_HOOK the same header serves the reference's own echo
// SERVER (tests/new-ws-echo/test_ws_server.cpp, compiled unchanged from its
// place, oracle/Makefile `refserver`): see the end of this file.
#pragma once
#include <cstddef>
#include <cstdint>

#ifndef FWS_REFCLIENT_CLIENTS
#define FWS_REFCLIENT_CLIENTS 1
#endif
#ifndef FWS_REFCLIENT_MSGS
#define FWS_REFCLIENT_MSGS 40000
#endif
#ifndef FWS_REFCLIENT_PORT
#define FWS_REFCLIENT_PORT 58600
#endif
#ifndef FWS_REFCLIENT_MSG_LEN
#define FWS_REFCLIENT_MSG_LEN 4096
#endif

namespace test {

inline constexpr const char *SERVER_IP = "127.0.0.1";
inline constexpr int SERVER_PORT = FWS_REFCLIENT_PORT;
inline constexpr size_t MAX_DATA_LEN = FWS_REFCLIENT_MSG_LEN;
// the client checks HashArr of the echoed payload every 16384 messages over all
// connections (test_ws_client.cpp:260), so a run needs more than 16384 in total
inline constexpr size_t MSG_LIMIT_PER_CLIENT = FWS_REFCLIENT_MSGS;
inline constexpr int REBORN_LIMIT_FOR_CLIENT = 1;
inline constexpr size_t CON_CLIENT_NUM = FWS_REFCLIENT_CLIENTS;
inline constexpr size_t TOTAL_MSG_CNT = MSG_LIMIT_PER_CLIENT * CON_CLIENT_NUM * REBORN_LIMIT_FOR_CLIENT;
inline constexpr int LISTEN_BACKLOG = 128;
inline constexpr bool ENABLE_TLS = false;
inline constexpr bool SHOULD_VERIFY_CERT = false;
inline constexpr const char *hostname = "";
inline constexpr const char *cert_file_path = "";
inline constexpr const char *key_file_path = "";
inline constexpr const char *ca_file_path = "";
inline constexpr const char *log_data_file_path = "./log_data.csv";

#define ENABLE_NO_DELAY 1

}  // namespace test

#ifdef FWS_REFSERVER_GPU_HOOK
// The one added line of gpu_floop.hpp's recipe (hook.Enable(ws_socket) before
// the listening socket goes to the loop), supplied without editing the server:
// this header is included after flashws.h / ws_server_socket.h / floop.h
// (test_ws_server.cpp:1-4), so a function-like macro on the name AddSocket
// touches only the server's own call, ctx.loop.AddSocket(std::move(ws_socket),
// ...) (test_ws_server.cpp:259), whose first argument passes through
// fws_amd_refserver::hooked(): GpuRxHook::Enable on the listening socket, then
// the same rvalue on to AddSocket. SIGTERM (the test's stop) prints the hook's
// GPU read count and exits.
#include <csignal>
#include <cstdio>
#include <unistd.h>
#include <utility>
#include "flashws_amd/gpu_floop.hpp"
namespace fws_amd_refserver {
inline fws_amd::GpuRxHookT<test::ENABLE_TLS> *g_hook = nullptr;
inline void on_term(int) {
    char b[64];
    const int k = std::snprintf(b, sizeof b, "gpu_reads %llu\n",
                                (unsigned long long)(g_hook ? g_hook->gpu_reads() : 0));
    if (k > 0) (void)!::write(1, b, (size_t)k);
    ::_exit(0);
}
template <class Sock>
Sock &&hooked(Sock &&listen) {
    static fws_amd::GpuContext gpu(0);
    static fws_amd::GpuRxHookT<test::ENABLE_TLS> hook(gpu);
    g_hook = &hook;
    hook.Enable(listen);
    std::signal(SIGTERM, on_term);
    std::printf("gpu hook enabled\n");
    std::fflush(stdout);
    return std::move(listen);
}
}  // namespace fws_amd_refserver
#define AddSocket(sock, ...) AddSocket(::fws_amd_refserver::hooked(sock), __VA_ARGS__)
#endif
