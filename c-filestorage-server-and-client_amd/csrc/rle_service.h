// rle_service.h — the resident small-call service shared by its kernel (rle_coop.hip svc_kernel)
// and the drop-in (rle_dropin.cpp): the mailbox layout in mapped host memory.
//
// The drop-in's small calls (one buffer of up to a few tens of KiB, already zero-copy: the kernel
// reads the caller's bytes from and writes its result into the thread's mapped buffer) spend most
// of their time on the launch, not on the codec: ~12 us per call with a polled completion against
// ~7 us when a resident kernel picks the request up from a mailbox (profiles/r4b_mailbox_probe.txt).
//
// One service per device serves every thread context (round 4, second form): kSvcGroups resident
// workgroups of kSvcWaves waves, launched once per busy period on one stream at the greatest
// priority, so that no other launch shares its hardware queue (a resident kernel holds every launch
// queued behind it on its queue: tools/probes/queue_probe.hip, profiles/r4n_queue_probe.txt; the
// first form, one workgroup per context on its own stream, let the contexts' services block each
// other's relaunches).  Each context owns a mailbox slot; workgroup g serves slots g, g + kSvcGroups,
// ...  Its wave 0 polls its slots' request lines (one 16-byte read per lane over PCIe, system-scope
// loads), the workgroup runs the cooperative codec body for a complete new request (rle_coop.hip
// enc_coop_body / dec_coop_body) on the slot's buffers, every wave releases its output at system
// scope and thread 0 stores the acknowledgement.  The workgroups leave together: kSvcIdleUs after
// the last request any of them served (a shared device-memory timestamp), kSvcLifeUs after the
// launch, or on the stop word; the first to decide raises `exiting`, the last out stores `gone`
// (the launch's generation).  A request that finds the service gone relaunches it.
#pragma once
#include <stdint.h>

namespace rle {

constexpr uint32_t kSvcWaves = 8;      // waves of a service workgroup (the cooperative bodies' widest form)
constexpr uint32_t kSvcGroups = 8;     // service workgroups
constexpr uint32_t kSvcPerGroup = 16;  // slots one workgroup polls (wave 0: 4 lanes x 16 bytes each)
constexpr uint32_t kSvcSlots = kSvcGroups * kSvcPerGroup;
constexpr uint32_t kSvcIdleUs = 1000;
constexpr uint32_t kSvcLifeUs = 20000;
constexpr uint32_t kSvcEncode = 0, kSvcDecode = 1;

// Request line of a slot (64 bytes): written by the host, the sequence number last (and `tail`
// just before it: a line whose tail differs from req is read again).
struct SvcReq {
    uint32_t req;        // sequence number of the latest request
    uint32_t op;         // kSvcEncode / kSvcDecode
    uint32_t in_len;     // encode: U; decode: C
    uint32_t out_len;    // decode: U
    uint32_t cap;        // decode: the output slot's capacity (U + E)
    uint32_t flags;      // bit 0: write-through output stores
    uint32_t rsv;
    uint32_t tail;       // = req once the line is complete
    uint64_t src;        // device address of the request's input (the context's mapped buffer)
    uint64_t dst;        // ... and of its output
    uint32_t pad[4];
};
// Acknowledgement line of a slot (64 bytes): written by the service.
struct SvcAck {
    uint32_t ack;        // sequence number of the latest served request
    uint32_t status;     // its RLE_STATUS_*
    uint64_t res_len;    // encode: C
    uint32_t pad[12];
};
struct SvcMail {
    SvcReq r;
    SvcAck a;
};
// The mapped region: the host's line (stop word, slots in use), the service's line (gone), then
// the slots.
struct SvcHead {
    uint32_t stop;       // nonzero: end the service now
    uint32_t nslots;     // slots 0 .. nslots-1 may hold requests
    uint32_t pad[14];
};
struct SvcGone {
    uint32_t gone;       // generation of the launch that has ended
    uint32_t pad[15];
};
struct SvcRegion {
    SvcHead head;
    SvcGone gone;
    SvcMail slot[kSvcSlots];
};
// Device-memory state of one launch (zeroed before it).
struct SvcState {
    uint64_t last;       // wall clock of the latest request served
    uint32_t exiting;    // set once: every workgroup leaves
    uint32_t exited;     // workgroups gone
};
static_assert(sizeof(SvcReq) == 64 && sizeof(SvcAck) == 64 && sizeof(SvcHead) == 64 && sizeof(SvcGone) == 64,
              "mailbox lines");

}  // namespace rle
