// rx_ring_variants.hip — timing variants of the receive-ring kernel
// (rx_ring.hip) that the product library does not carry, for
// tools/rx_ring_probe.py.  rxv_launch(geo, stream, k):
//   0 the product shape <13, default line 0, nt rest, 4 waves/WG>
//   1 every line default policy      2 every line nontemporal
//   3 2 waves/WG   4 8 waves/WG   5 1 wave/WG
//   6 16 lines per batch   7 8 lines per batch (two batches for 1500 B)
//   8 the product shape with a 6-waves/SIMD register floor
//   9 12 lines per batch
//  10 every chunk range-checked (F = 0: round 5's first product shape)
//  11 F with 8 lines per batch
//  12 / 13 line 0 / lines 0-1 loaded before the slot's length arrives
//  14 the product shape with each group's lines >= 2 in a rotated order
//  20-23 buffer lists (LIST = 1, g.off set): the product shape, then lines
//        >= 1 with the policy nt sc1 / default / sc1 instead of nt
//  24-29 buffer lists with each packet's last line at the default policy
//        (LL), the other lines >= 1 nt / nt sc1 / sc0 nt / sc0 sc1 /
//        sc0 nt sc1 / sc0
// Every variant computes the same verdicts and sums.  Not part of the ABI.
#include "../netstack_amd/csrc/rx_ring.hip"

extern "C" int rxv_launch(const nsk::RxGeo* g, void* stream, int k) {
  hipStream_t s = (hipStream_t)stream;
  switch (k) {
    case 1: return (int)nsk::launch_rx_ring_t<13, 0, 0>(*g, s);
    case 2: return (int)nsk::launch_rx_ring_t<13, 2, 2>(*g, s);
    case 3: return (int)nsk::launch_rx_ring_t<13, 0, 2, 2>(*g, s);
    case 4: return (int)nsk::launch_rx_ring_t<13, 0, 2, 8>(*g, s);
    case 5: return (int)nsk::launch_rx_ring_t<13, 0, 2, 1>(*g, s);
    case 6: return (int)nsk::launch_rx_ring_t<16>(*g, s);
    case 7: return (int)nsk::launch_rx_ring_t<8>(*g, s);
    case 8: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 6>(*g, s);
    case 9: return (int)nsk::launch_rx_ring_t<12>(*g, s);
    case 10: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 0>(*g, s);
    case 11: return (int)nsk::launch_rx_ring_t<8, 0, 2, 4, 1, 1>(*g, s);
    case 12: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 1>(*g, s);
    case 13: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 2>(*g, s);
    case 14: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 0, 0, 1>(*g, s);
    case 20: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 0, 1>(*g, s);
    case 21: return (int)nsk::launch_rx_ring_t<13, 0, 18, 4, 1, 1, 0, 1>(*g, s);
    case 22: return (int)nsk::launch_rx_ring_t<13, 0, 0, 4, 1, 1, 0, 1>(*g, s);
    case 23: return (int)nsk::launch_rx_ring_t<13, 0, 16, 4, 1, 1, 0, 1>(*g, s);
    case 24: return (int)nsk::launch_rx_ring_t<13, 0, 2, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 25: return (int)nsk::launch_rx_ring_t<13, 0, 18, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 26: return (int)nsk::launch_rx_ring_t<13, 0, 3, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 27: return (int)nsk::launch_rx_ring_t<13, 0, 17, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 28: return (int)nsk::launch_rx_ring_t<13, 0, 19, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    case 29: return (int)nsk::launch_rx_ring_t<13, 0, 1, 4, 1, 1, 0, 1, 0, 1>(*g, s);
    default: return (int)nsk::launch_rx_ring_t<13>(*g, s);
  }
}
