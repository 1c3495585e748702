// Native checkpoint / restart (runtime/checkpoint.cpp): the Python driver's
// on-disk format (utils/checkpoint.py), so either driver resumes the other's
// checkpoints on any rank count.
#pragma once

#include <string>

#include "heat2d/runtime.hpp"

namespace heat2d {
namespace ckpt {

struct Meta {
  int64_t step = 0;
  int nranks = 1;
  int dtype = 1;  // 0 fp32, 1 fp64
  int64_t n_owned = 0, n_input = 0;
  std::string convention = "ghost";  // ghost | inclusive
  double sigma = 0, nu = 0, dom_len = 0, r = 0;
  int64_t edge_shift = 0;  // the writer's decomposition (common.hpp decompose); absent in older saves: 0
  std::string dir;  // read_meta: the directory holding this step's files
};

// Layout (v2): DIR/step-NNNNNNNNNNNN[-G]/{rankNNNNN.npy, meta.json} +
// DIR/latest, a one-line pointer to the newest COMPLETE step directory.
// Collective use: every rank picks the same FRESH step directory
// (step_dir_name, then a barrier before anyone creates it: a step saved again —
// a restart at its final step, a re-run into the same directory — gets a new
// generation -G instead of overwriting files `latest` may point at), writes
// and fsyncs its slab there; after a barrier rank 0 writes meta.json there,
// fsyncs it and the directory, republishes DIR/latest (temp file + fsync +
// rename, atomic) and prunes all but the two newest step directories. A crash
// at any point leaves `latest` on a complete checkpoint; rank files of two
// steps can never be mixed. read_meta also accepts a step directory itself
// and the v1 flat layout (DIR/meta.json + DIR/rank*.npy).
std::string step_dir_name(const std::string& dir, int64_t step);
void write_rank(const std::string& dir, const std::string& name, int rank, Solver& s);
void write_meta(const std::string& dir, const std::string& name, const Meta& m);
Meta read_meta(const std::string& dir);
// Global rows [row0, row0 + nrows) x ncols of the checkpointed field into `out`
// (row-major, ld = ncols), gathered from however many writer files there are
// (their shapes checked against the writer's decomposition).
void read_rows(const Meta& m, int64_t row0, int64_t nrows, int64_t ncols, int dtype, void* out);

}  // namespace ckpt
}  // namespace heat2d
