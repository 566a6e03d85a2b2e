// rle_service.h — the resident small-call service shared by its kernel (rle_coop.hip svc_kernel)
// and the drop-in (rle_dropin.cpp): the mailbox layout in mapped host memory.
//
// The drop-in's small calls (one buffer of up to a few tens of KiB, already zero-copy: the kernel
// reads the caller's bytes from and writes its result into the thread's mapped buffer) spend most
// of their time on the launch, not on the codec: ~12 us per call with a polled completion against
// ~7 us when a resident kernel picks the request up from a mailbox (profiles/r4b_mailbox_probe.txt).
// The service gives each thread context its own resident workgroup (kSvcWaves waves, on the
// context's own service stream): the host writes the request into the context's mailbox line and
// bumps its sequence number; wave 0 polls the line (one 64-byte read over PCIe per poll: request,
// sizes and stop word together), the workgroup runs the cooperative codec body for it
// (rle_coop.hip enc_coop_body / dec_coop_body, barrier-uniform form), every wave releases its
// output at system scope and thread 0 stores the acknowledgement.  The workgroup ends by itself
// kSvcIdleUs after its last request (and at most kSvcLifeUs after its launch; the stop word ends it
// at process exit), marking `gone` with its launch generation; a request that finds it gone
// relaunches it.
#pragma once
#include <stdint.h>

namespace rle {

constexpr uint32_t kSvcWaves = 8;     // waves of a service workgroup (the cooperative bodies' widest form)
constexpr uint32_t kSvcIdleUs = 1000;
constexpr uint32_t kSvcLifeUs = 20000;
constexpr uint32_t kSvcEncode = 0, kSvcDecode = 1;

// Host line (64 bytes, one read per poll): written by the host, the sequence number last (and
// `tail` just before it: a line whose tail differs from req is read again).
struct SvcReq {
    uint32_t req;        // sequence number of the latest request
    uint32_t op;         // kSvcEncode / kSvcDecode
    uint32_t in_len;     // encode: U; decode: C
    uint32_t out_len;    // decode: U
    uint32_t cap;        // decode: the output slot's capacity (U + E)
    uint32_t flags;      // bit 0: write-through output stores
    uint32_t stop;       // nonzero: end the service now
    uint32_t tail;       // = req once the line is complete
    uint32_t pad[8];
};
// Device line (64 bytes): written by the service.
struct SvcAck {
    uint32_t ack;        // sequence number of the latest served request
    uint32_t status;     // its RLE_STATUS_*
    uint64_t res_len;    // encode: C
    uint32_t gone;       // generation of the launch that has ended
    uint32_t pad[11];
};
struct SvcMail {
    SvcReq r;
    SvcAck a;
};
static_assert(sizeof(SvcReq) == 64 && sizeof(SvcAck) == 64, "mailbox lines");

}  // namespace rle
