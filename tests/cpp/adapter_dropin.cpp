// Compile/link check: the MI355X decoder drops into flashws's own types.
// Built against the reference headers in the build container only
// (tests/test_adapter_cpu.py); never run (no GPU there).
#include "flashws/flashws.h"
#include "flashws_amd/gpu_ws.hpp"

#include <cstdio>

namespace {

struct EchoSink {                      // shape of tests/new-ws-echo's SetOnRead handler
    size_t bytes = 0, msgs = 0;
    void on_read(uint32_t opcode, fws::IOBuffer &&buf, bool frame_end, bool msg_end, bool is_ctl) {
        (void)opcode; (void)frame_end; (void)is_ctl;
        bytes += (size_t)buf.size;
        msgs += msg_end;
    }
    void on_ping(std::string_view p) { bytes += p.size(); }
    void on_close(uint32_t code, std::string_view p) { (void)code; (void)p; }
    fws::IOBuffer request_buf(size_t n) { return fws::RequestBuf(n); }
};

}  // namespace

int main() {
    fws_amd::GpuContext ctx(0, 1 << 16, 1 << 22);
    fws_amd::GpuRxDecoder<fws::IOBuffer> rx(ctx);
    fws::IOBuffer io = fws::RequestBuf(64 + 32);
    io.start_pos = 32;
    const uint8_t hello[] = {0x81, 0x85, 0x37, 0xfa, 0x21, 0x3d, 0x7f, 0x9f, 0x4d, 0x51, 0x58};
    memcpy(io.data + 32, hello, sizeof(hello));
    io.size = sizeof(hello);
    EchoSink sink;
    int r = rx.OnRecvData(io, sink);
    std::printf("ret=%d bytes=%zu msgs=%zu\n", r, sink.bytes, sink.msgs);
    // echo the payload back as a client-masked BIN frame: WriteFrame's
    // arguments with flashws's own WSTxFrameType (net/w_socket.h:25-31)
    fws_amd::GpuTxEncoder tx(ctx, /*is_server=*/false);
    tx.Queue(io.data + 32 + 6, 5, fws::WS_BIN_FRAME, true, 0x3d21fa37u);
    std::vector<uint8_t> wire;
    r |= tx.Flush(wire);
    std::printf("tx bytes=%zu\n", wire.size());
    int dev_count = 0;
    fws_gpu_device_count(&dev_count);
    return r;
}
