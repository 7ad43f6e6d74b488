// L3-domain pairing of loopback connections (in-process broker and consumers).
//
// Each consumer connection's receiving thread (an engine source thread) is pinned to one L3
// domain (one CCD of an EPYC socket: 8 cores sharing 32 MB of L3), round robin over the domains
// of its affinity mask, and registers the connection's local port. The embedded broker's thread
// that serves that connection looks its peer port up and pins itself to the same domain. The
// broker's copy of a fetch response into the socket buffer then lands in the L3 that the
// receive copy reads: 19.8 GB/s per receiving core with the pair on one CCD against 12.9 GB/s
// across two (profiles/r5_llc_pair.jsonl, csrc/tests/recv_bounce_bench.cpp). That holds for a
// copying sender only: bench.py's broker splices the stored batches (zero copy), so the receive
// copy reads DRAM either way, and in the pipeline the pairing measured no gain (same file). It
// is opt-in, for a broker that copies.
//
// Only meaningful when broker and consumers share a process (bench.py, the tests); a remote
// broker simply never finds a registration. GALE_LLC_PAIR=1 turns it on.
#pragma once

namespace gale {
namespace llc {

bool enabled();
// Pins the calling thread to the next L3 domain (round robin) of its current affinity mask.
// Returns the domain's lowest CPU id, or -1 (no sysfs cache topology, or a single domain).
int pin_self_next_domain();
// Client side: the connection with this local port is read by the calling thread; registered
// only when that thread was pinned by pin_self_next_domain().
void register_local_port(int local_port);
// Broker side: pins the calling thread to the domain registered for this peer port. Returns
// true once pinned (false: nothing registered for it, yet or at all).
bool pin_self_for_peer(int peer_port);

}  // namespace llc
}  // namespace gale
