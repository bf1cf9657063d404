// Internal glue: public ABI structs, error handling.
#pragma once
#include <exception>
#include <stdexcept>
#include <string>

#include "../../include/ocf.h"
#include "ocf_common.h"

namespace ocf {
using ScatterArgs = OcfScatterArgs;
void set_error(const std::string& msg);
// Faults a kernel detects without stopping (ocf_gemm_pair's bounded hand-off wait) are written to a
// pinned, host-coherent word; every entry point reports a pending one (once) before doing anything.
uint32_t* async_error_word();        // device-visible address of the word (allocated on first use)
void check_async_errors();
extern int g_mlp_max_polls;          // ocf_mlp_step's barrier wait (ocf_set_tuning "mlp_max_polls")
extern int g_encdec_max_polls;       // ocf_gather_encdec's wait (ocf_set_tuning "encdec_max_polls")
extern int g_encdec_rowres;          // ocf_gather_encdec's row-resident form (ocf_set_tuning "encdec_rowres")
// a feature rank's gathers as row-resident launches (ocf_sparse.hip; ocf_rank_step phases 0 / 1): false = not
// applicable, nothing launched
bool rank_rowres_enc(const OcfGatherArgs& e, const OcfRowsReduceArgs& r, hipStream_t s);
bool rank_rowres_dec(const OcfBiasActArgs& hb, const OcfGatherArgs& d, const OcfRowsReduceArgs& r, hipStream_t s);
extern int g_enc_tiles_pack;         // ocf_encoder_tiles' pre-pass (ocf_set_tuning "enc_tiles_pack")
// The encoder -> decoder hand-off's gate (ocf_gather_encdec): a device word a decoder chunk that gave up sets to
// its launch's generation; the row-stream weight-update launches issued after that encdec launch (the same
// generation) read it at entry and write nothing when it matches.  The generation only grows (never 0), so no
// launch has to clear the word.
uint32_t* encdec_gate_word();        // device word (allocated on first use), nullptr before any encdec launch
uint32_t encdec_generation();        // the generation of the last encdec launch issued (0: none)
uint32_t next_encdec_generation();   // a new generation for an encdec launch being issued
}  // namespace ocf

#define OCF_TRY_BEGIN try { ocf::check_async_errors();
#define OCF_TRY_END                                       \
  return 0;                                               \
  }                                                       \
  catch (const std::exception& e) {                       \
    ocf::set_error(e.what());                             \
    return 1;                                             \
  }

#define OCF_CHECK(cond, msg)                              \
  do {                                                    \
    if (!(cond)) throw std::runtime_error(msg);           \
  } while (0)

#define OCF_HIP(expr)                                                               \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + \
                               " at " __FILE__ ":" + std::to_string(__LINE__));     \
  } while (0)
