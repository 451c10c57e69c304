// tx_variants.hip — timing variants of the structured TX kernel (tcp_tx.hip)
// that the product library does not carry, for tools/tx_struct_probe.py:
//   txv_launch(geo, stream, k): 0 = production shape, 1 = no segment
//   reductions (wrong sums), 2 = 8 windows in flight, 3 = 4 windows in
//   flight, 4 = production without the header write-back (fields unwritten),
//   5 = neither reductions nor write-back (the bare stream + header reads),
//   6 = 12 windows in flight, 7 = 6 without the write-back; 8 / 9 / 10 = the
//   two-pass shape (g->xs set) with 12 / 16 / 8 windows in flight; 11 = the
//   two passes with no header write-back (fields unwritten); 12 / 13 / 14 =
//   the two passes with the persistent header pass at 4 / 16 / 2 waves per CU
//   (the product runs 24); 15 = the two passes, one-shot header pass;
//   16 / 17 = the persistent header pass at 24 / 32 waves per CU.
// Not part of the product ABI.
#include "../netstack_amd/csrc/tcp_tx.hip"

extern "C" int txv_launch(const nsk::TxGeo* g, void* stream, int k) {
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (k) {
    case 1: e = nsk::launch_tcp_tx_t<16, 2, 0, 2>(*g, s); break;
    case 2: e = nsk::launch_tcp_tx_t<8, 2, 0, 1>(*g, s); break;
    case 3: e = nsk::launch_tcp_tx_t<4, 2, 0, 1>(*g, s); break;
    case 4: e = nsk::launch_tcp_tx_t<16, 2, 0, 1, 1>(*g, s); break;
    case 5: e = nsk::launch_tcp_tx_t<16, 2, 0, 2, 1>(*g, s); break;
    case 6: e = nsk::launch_tcp_tx_t<12, 2, 0, 1>(*g, s); break;
    case 7: e = nsk::launch_tcp_tx_t<12, 2, 0, 1, 1>(*g, s); break;
    case 8: e = nsk::launch_passes<12, 2, 0, 1>(*g, s); break;
    case 9: e = nsk::launch_passes<16, 2, 0, 1>(*g, s); break;
    case 10: e = nsk::launch_passes<8, 2, 0, 1>(*g, s); break;
    case 11: {  // the two passes, the header pass without its write-back (timing only)
      nsk::TxGeo h = *g;
      h.tile = g->htile;
      e = nsk::launch_tcp_tx_t<16, 2, 0, 1, 0, 1>(*g, s);
      if (e == hipSuccess) e = nsk::launch_tcp_tx_t<16, 2, 0, 1, 1, 2>(h, s);
      break;
    }
    case 12: e = nsk::launch_passes<16, 2, 0, 1, 1>(*g, s, 4); break;
    case 13: e = nsk::launch_passes<16, 2, 0, 1, 1>(*g, s, 16); break;
    case 14: e = nsk::launch_passes<16, 2, 0, 1, 1>(*g, s, 2); break;
    case 15: e = nsk::launch_passes<16, 2, 0, 1, 0>(*g, s); break;
    case 16: e = nsk::launch_passes<16, 2, 0, 1, 1>(*g, s, 24); break;
    case 17: e = nsk::launch_passes<16, 2, 0, 1, 1>(*g, s, 32); break;
    default: e = nsk::launch_tcp_tx_t<16, 2, 0, 1>(*g, s); break;
  }
  return (int)e;
}
