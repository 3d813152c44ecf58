#pragma once
namespace hf2d {
// q = hf_div(a, b), s = hf_sqrt(a) on the GPU (host arrays of n doubles)
void div_probe(const double* a, const double* b, double* q, double* s, long n);
}  // namespace hf2d
