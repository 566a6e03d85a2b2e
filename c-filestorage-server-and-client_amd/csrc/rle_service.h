// rle_service.h — the resident small-call service shared by its kernel (rle_coop.hip svc_kernel)
// and the drop-in (rle_dropin.cpp): the mailbox layout in mapped host memory.
//
// The drop-in's small calls (one buffer of up to a few tens of KiB, already zero-copy: the kernel
// reads the caller's bytes from and writes its result into the thread's mapped buffer) spend most
// of their time on the launch, not on the codec: ~12 us per call with a polled completion
// (profiles/r4a_sync_probe.txt) against a few us of work.  The service is one kernel that stays
// resident while calls keep coming: each thread context owns a mailbox slot, posts a request by
// writing its descriptor and bumping req[slot], and polls ack[slot]; a workgroup of the service
// claims the slot's request (an atomic on the claim word in device memory: any workgroup may
// serve any slot), runs the cooperative codec body for it (rle_coop.hip enc_coop_body /
// dec_coop_body, barrier-uniform form) and acknowledges it behind a system-scope release of every
// output byte.  The service ends by itself after kSvcIdleUs without a request anywhere (and at most
// kSvcLifeUs after its launch; a stop word ends it at process exit), each workgroup marking gone[g]
// with the launch's generation; a request that finds every workgroup gone relaunches it.
#pragma once
#include <stdint.h>

namespace rle {

constexpr uint32_t kSvcSlots = 64;    // mailboxes: one per thread context (wave 0 polls one per lane)
constexpr uint32_t kSvcGroups = 4;    // workgroups of the service
constexpr uint32_t kSvcWaves = 8;     // waves per workgroup (the cooperative bodies' widest form)
constexpr uint32_t kSvcIdleUs = 1000;
constexpr uint32_t kSvcLifeUs = 20000;
constexpr uint32_t kSvcEncode = 0, kSvcDecode = 1;

struct SvcDesc {            // one request: written by the host before it bumps req[slot]
    uint64_t src, dst;      // device addresses (the context's mapped buffer)
    uint64_t in_len;        // encode: U; decode: C
    uint64_t out_len;       // decode: U
    uint64_t cap;           // decode: the output slot's capacity (U + E)
    uint32_t op;            // kSvcEncode / kSvcDecode
    uint32_t flags;         // launch flags (bit 0: write-through stores)
    uint64_t res_len;       // device: encode C
    uint32_t res_status;    // device: RLE_STATUS_*
    uint32_t pad[5];
};
static_assert(sizeof(SvcDesc) == 80, "SvcDesc layout");

struct SvcBox {
    uint32_t req[kSvcSlots];     // host: the slot's latest request sequence number
    uint32_t ack[kSvcSlots];     // device: the slot's latest served sequence number
    uint32_t gone[kSvcGroups];   // device: the generation whose workgroup g has ended
    uint32_t stop;               // host: nonzero ends the service at its next poll
    uint32_t pad[15 - kSvcGroups];
    SvcDesc desc[kSvcSlots];
};

}  // namespace rle
