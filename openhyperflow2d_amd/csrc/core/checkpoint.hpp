// .hf2d checkpoint: raw x-major image of 1248-byte CellRecords, byte
// compatible with the reference's swap file (obj_data/obj_data.cpp:117-319,
// deeps2d_core.cpp:1816-1849).  GlobalTime is stored in cell (0,0).time.
// An optional JSON sidecar (<file>.meta) records what the raw image cannot
// (iteration counter, dt, solver version) without touching the layout.
#pragma once

#include <string>

#include "case.hpp"

namespace hf2d {

// Returns true and fills J when `path` exists with exactly nx*ny*1248 bytes.
bool read_hf2d(const std::string& path, Field& J);
// Windowed field (Field::resize_window): the resident columns' slab at its
// file offset plus the CT / TurbType words of every other cell (streamed in
// blocks, nothing else of them is kept).  False unless the size matches.
bool read_hf2d_window(const std::string& path, Field& J);
// one record (i, j) of an image of nx*ny records
bool read_hf2d_record(const std::string& path, int nx, int ny, int i, int j, CellRecord& out);
// zero-filled image of the full size (the reference's swap file of a cold start)
void create_zero_hf2d(const std::string& path, int nx, int ny);
// a file of exactly nx*ny records exists at path
bool checkpoint_image_present(const std::string& path, int nx, int ny);
// Writes the whole field (pwrite in <=1 GiB chunks).
void write_hf2d(const std::string& path, const Field& J);
// Writes a column slab [i0, i1) of a global-size file at its file offset
// (per-rank checkpoint without a gather).
void write_hf2d_slab(const std::string& path, const Field& local, int local_i0, int global_i0, int ncols,
                     int global_nx);
void write_meta(const std::string& path, long iteration, double dt, double time);
bool read_meta(const std::string& path, long& iteration, double& dt, double& time);

}  // namespace hf2d
