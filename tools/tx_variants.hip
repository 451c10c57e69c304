// tx_variants.hip — timing variants of the structured TX kernel (tcp_tx.hip)
// that the product library does not carry, for tools/tx_struct_probe.py:
//   txv_launch(geo, stream, k): 0 = production shape, 1 = no segment
//   reductions at all (timing only: wrong sums), 2 = 32 windows in flight,
//   3 = 4 windows in flight, 4 = the header path alone with 2-byte stores.
// Not part of the product ABI.
#include "../netstack_amd/csrc/tcp_tx.hip"

extern "C" int txv_launch(const nsk::TxGeo* g, void* stream, int k) {
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  switch (k) {
    case 1: e = nsk::launch_tcp_tx_t<16, 2, 0, 2>(*g, s); break;
    case 2: e = nsk::launch_tcp_tx_t<32, 2, 0, 1>(*g, s); break;
    case 3: e = nsk::launch_tcp_tx_t<4, 2, 0, 1>(*g, s); break;
    default: e = nsk::launch_tcp_tx_t<16, 2, 0, 1>(*g, s); break;
  }
  return (int)e;
}
