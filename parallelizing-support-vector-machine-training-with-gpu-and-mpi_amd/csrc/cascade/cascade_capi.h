// Helpers shared by the C ABIs of the cascade (CPU group in libsvm355_core, device groups and
// ranks in libsvm355_hip).
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "cascade.h"

namespace svm355 {

CascadeConfig config_from(const svm_cascade_cfg* c);
// Builds the C result from rank outputs (outs[0] = the lowest rank this call drove; it provides
// the model); B0 is that rank's backend (for the SV rows).
svm_cascade_out* build_cascade_out(const std::vector<const CascadeOutput*>& outs, Backend& B0, int world,
                                   int first_rank, const char* transport, const char* backend);
// Row-major host rows of rank r's partition (contiguous ceil(n / P) chunks) and their global ids.
std::vector<int64_t> partition_ids(int64_t n, int P, int r, int64_t* lo, int64_t* hi);

// A rank over caller-supplied host collectives (hostcomm.cpp).  staging null: the buffers handed to
// the transport are host memory; else they are `staging`'s memory (device) and travel through host
// copies.  The callbacks must stay valid for the transport's lifetime.
bool host_comm_valid(const svm_host_comm* c);
std::unique_ptr<Transport> make_hostcomm_transport(const svm_host_comm& c, Backend* staging);

// Transport exerciser (exercise.cpp): runs this rank's op list of `script` with checked payloads;
// throws TransportError naming the rank, the op and what differed.
void exercise_transport(Transport& t, Backend& B, const std::string& script);
// Every op the cascade driver issues over P ranks (tree pairs per level included), bulk payloads of
// bulk_bytes: the RCCL preflight of the device groups and ranks.
std::string preflight_script(int P, int64_t bulk_bytes);

}  // namespace svm355
