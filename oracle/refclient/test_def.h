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
