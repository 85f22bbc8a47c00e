/*
 * group_plan.h — the order of one frame's device operations in a wcpt_group (include/wcpt.h wcpt_group_render;
 * executed by wcpt_group.hip). Pure C++ with no HIP types, so the ordering rules can be checked on a CPU:
 * tests/test_group_plan.py runs these plans through a stream/event simulation with random durations.
 *
 * Each local rank has a render stream (its context's) and, in a group of more than one, a communication stream; per
 * rank and payload buffer b two events: ready[b] (the render that wrote payload b has finished) and sent[b] (the
 * transfer that read payload b has finished). A frame, after every rank's arguments were validated:
 *   1. every sender that will rewrite payload b first makes its render stream wait for sent[b] (the previous transfer
 *      that read it), then points its next render at payload b (the root renders into its rows of the frame);
 *   2. every rank renders its row block;
 *   3. with presenting on: ready[b] is recorded behind each render, and each sender's communication stream waits for it
 *      (overlap on) -- or the transfers stay on the render streams (overlap off);
 *   4. the transfers: each sender sends payload b to the root and the root receives every other rank's block into its
 *      rows of the frame (RCCL: one ncclGroupStart/ncclGroupEnd around all of them), or each sender copies payload b
 *      into the root's frame (COPY transport: peer copies, no receive);
 *   5. interleaved row stripes (WCPT_GROUP_OPTION_ROW_STRIPE) with RCCL: the root received each block into a staging
 *      buffer, and now copies each one's stripes to their rows of the frame on the same stream (after the whole
 *      ncclGroupStart/End, so one host thread can post every rank's transfers of the frame in one group);
 *   6. sent[b] is recorded behind each sender's transfer.
 * The buffer index alternates between frames with overlap on (b = frame % 2), so frame k + 1 renders while frame k's
 * transfer is in flight; with overlap off it is always 0, and the transfer is in line with the renders.
 * DIRECT transport: every sender's render writes its block straight into the root's frame over xGMI (its gather output
 * is set once, at the frame's rows on the root device), so the frame is only the renders: no payload, event or
 * transfer step, and the presented frame is complete when the renders are.
 */
#pragma once

#include <cstdint>
#include <vector>

namespace wcpt {
namespace plan {

constexpr int kPayloadBuffers = 2;

enum Op : int32_t {
    kWaitSent = 0,      /* render stream waits for sent[buffer]: payload `buffer` is about to be rewritten      */
    kSetOutput = 1,     /* the rank's next render writes payload `buffer` (senders only)                        */
    kRender = 2,        /* the rank renders its row block on its render stream                                  */
    kRecordReady = 3,   /* ready[buffer] recorded on the render stream                                          */
    kCommWaitReady = 4, /* the communication stream waits for ready[buffer]                                     */
    kSend = 5,          /* payload `buffer` to `peer` (the root): RCCL send, or a peer copy into the root's frame */
    kRecv = 6,          /* the root receives rank `peer`'s block into its frame (RCCL only)                     */
    kRecordSent = 7,    /* sent[buffer] recorded behind the rank's transfer                                     */
    kScatter = 8,       /* the root copies rank `peer`'s received stripes from staging to their frame rows        */
};

enum Stream : int32_t { kRenderStream = 0, kCommStream = 1 };

/* wcpt.h WCPT_GROUP_TRANSPORT_* */
enum Transport : int32_t { kRccl = 0, kCopy = 1, kDirect = 2 };

struct Step {
    int32_t op, rank, buffer, peer, stream;
};

/* What the plan needs of a local rank: its number and which payload buffers have a recorded sent event. */
struct RankState {
    int32_t rank;
    bool sent_pending[kPayloadBuffers];
};

inline int payload_buffer(bool overlap, uint64_t frame) { return overlap ? (int)(frame % kPayloadBuffers) : 0; }

/* The steps of frame `frame` for this process's ranks (`local`, in rank order), in issue order; marks sent[b] pending
 * for every sender whose transfer was planned. `exchange`: presenting with more than one rank. */
inline void frame_steps(int nranks, int root, bool overlap, bool exchange, int transport, uint64_t frame,
                        std::vector<RankState>& local, std::vector<Step>& out, bool stripes = false)
{
    out.clear();
    const bool copy = transport == kCopy;
    if (transport == kDirect) exchange = false; /* the renders are the exchange */
    const int b = payload_buffer(overlap, frame);
    if (exchange) {
        for (const RankState& lr : local) {
            if (lr.rank == root) continue;
            if (lr.sent_pending[b]) out.push_back({kWaitSent, lr.rank, b, -1, kRenderStream});
            out.push_back({kSetOutput, lr.rank, b, -1, kRenderStream});
        }
    }
    for (const RankState& lr : local) out.push_back({kRender, lr.rank, b, -1, kRenderStream});
    if (!exchange) return;
    const int xs = overlap ? kCommStream : kRenderStream;
    for (const RankState& lr : local) {
        if (lr.rank == root) continue;
        out.push_back({kRecordReady, lr.rank, b, -1, kRenderStream});
        if (overlap) out.push_back({kCommWaitReady, lr.rank, b, -1, kCommStream});
    }
    for (const RankState& lr : local) {
        if (lr.rank != root) {
            out.push_back({kSend, lr.rank, b, root, xs});
            continue;
        }
        if (copy) continue; /* the senders write the root's rows themselves */
        for (int r = 0; r < nranks; r++)
            if (r != root) out.push_back({kRecv, lr.rank, b, r, xs});
    }
    if (stripes && !copy)
        for (const RankState& lr : local)
            if (lr.rank == root)
                for (int r = 0; r < nranks; r++)
                    if (r != root) out.push_back({kScatter, lr.rank, b, r, xs});
    for (RankState& lr : local) {
        if (lr.rank == root) continue;
        out.push_back({kRecordSent, lr.rank, b, -1, xs});
        lr.sent_pending[b] = true;
    }
}

} // namespace plan
} // namespace wcpt
