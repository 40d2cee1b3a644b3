/**
 * @file lora_phy/ChirpGenerator.hpp
 * Header-only chirp generator with the semantics of the reference's
 * genChirp (/root/reference/include/lora_phy/ChirpGenerator.hpp:24-51):
 * a float frequency ramp from fMin+f0 in steps of 2*pi*bw_scale/(N*osr^2),
 * wrapped at fMax, integrated into a running phase, one polar() sample per
 * step; the accumulator is finally wrapped to [0, 2*pi) in double precision
 * (the reference's unqualified floor() on a float resolves to ::floor(double)).
 * Callers use it to build the down-chirp for the external dechirp in front
 * of lora_demodulate(); bit-identical output keeps that chain in parity.
 */
#pragma once

#include <cmath>
#include <complex>

#include <lora_phy/phy.hpp>

template <typename Type>
int genChirp(std::complex<Type>* samps, int N, int osr, int NN, Type f0, bool down,
             const Type ampl, Type& phaseAccum, Type bw_scale = Type(1)) {
    const Type lo = -lora_phy::PI * bw_scale / osr;
    const Type hi = lora_phy::PI * bw_scale / osr;
    const Type inc = (2 * lora_phy::PI * bw_scale) / (N * osr * osr);
    const Type sgn = down ? Type(-1) : Type(1);
    float freq = lo + f0;
    int n = 0;
    for (; n < NN; ++n) {
        freq += inc;
        if (freq > hi) freq -= (hi - lo);
        if (sgn < 0) phaseAccum -= freq; else phaseAccum += freq;
        samps[n] = std::polar(ampl, phaseAccum);
    }
    const double turns = std::floor(static_cast<double>(phaseAccum / (2 * lora_phy::PI)));
    phaseAccum = static_cast<Type>(static_cast<double>(phaseAccum) - turns * 2 * lora_phy::PI);
    return n;
}
