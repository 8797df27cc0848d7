/*
 * flacgen.h -- seeded synthetic FLAC writer (test / benchmark input generator).
 *
 * Writes complete FLAC streams (fLaC + STREAMINFO [+ extra metadata] + frames with
 * CRC-8/CRC-16 and a correct STREAMINFO MD5) from synthetic PCM, inside zflac's
 * defined input domain. The source PCM it returns is ground
 * truth: generator -> oracle and generator -> HIP path must reproduce it exactly.
 * This is the repository's own encoder; it is not derived from libFLAC or zflac.
 */
#ifndef FLACGEN_H
#define FLACGEN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { FG_VERBATIM = 0, FG_FIXED = 2, FG_LPC = 3 };

typedef struct flacgen_config {
    int channels;          /* 1..8 */
    int bps;               /* 4..32 */
    int block_size;        /* nominal block size (16..65535) */
    int predictor;         /* FG_VERBATIM / FG_FIXED / FG_LPC */
    int order;             /* fixed: 0..4, lpc: 1..32 */
    int precision;         /* lpc coefficient precision, 1..15 */
    int max_shift;         /* cap on the lpc shift (0..15) */
    int stereo_mode;       /* 1 = L/R, 8 = left/side, 9 = side/right, 10 = mid/side, -1 = per-frame best */
    int partition_order;   /* requested rice partition order (clamped per frame) */
    int rice_k;            /* -1 = best per partition, else forced parameter */
    int rice2;             /* 1 = always code residuals with the 5-bit (Rice2) parameter */
    int escape_every;      /* every Nth partition (globally counted) is escape-coded; 0 = never */
    int wasted_bits;       /* PCM has this many zero LSBs */
    int sample_rate;
    int variable_blocking; /* 1 = blocking-strategy bit set, sample-number coding, random block sizes */
    int write_total;       /* 1 = STREAMINFO total samples set, 0 = unknown (0) */
    int extra_metadata;    /* 1 = add PADDING, APPLICATION, SEEKTABLE, VORBIS_COMMENT blocks */
    int verbatim_every;    /* every Nth subframe verbatim; 0 = never */
    int silence_every;     /* every Nth frame, channel 0 is digital silence; 0 = never */
    int rate_code_mode;    /* 0 = table code when possible, 1 = 16-bit Hz, 2 = Hz/10, 3 = from STREAMINFO */
    double tone_amp;       /* total tone amplitude, fraction of full scale */
    double noise_lsb;      /* rms of the white-noise floor, in significant LSBs */
    double stereo_corr;    /* R = corr * L + noise */
    int fault_frame;       /* frame index to corrupt, -1 = none */
    int fault_kind;        /* 1 reserved subframe type, 2 residual method 2, 3 LPC precision code 15,
                              4 that frame has block size 1, 5 partition order not dividing the block,
                              6 channel-0 subframe pinned to the SampleType maximum (stereo: the
                              decorrelated output overflows), 7 LPC with the largest coefficients of
                              the precision (decodable when the signal is quiet), 8 same but written
                              even when zflac's InterType sums overflow */
    uint64_t n_samples;    /* per channel */
    uint64_t seed;
    /* --- parity-edge options (all 0 = off) --- */
    int dual_mono_every;   /* every Nth frame (f % N == N - 1) R = L - dual_mono_offset: constant side */
    int dual_mono_offset;
    int const_side;        /* constant side subframes: 0 never (coded as fixed/verbatim), 1 zflac width
                              (bits_per_sample - wasted, src/zflac.zig:447), 2 RFC width (bps + 1 - wasted) */
    int plant_sync_every;  /* every Nth frame (f % N == N - 1), channel 0 is verbatim and carries a copy
                              of the frame's own CRC-8-valid header inside its sample data (bps 8 / 16 /
                              24, independent channels only) */
    int allow_side_overflow; /* 1 = write side channels that do not fit the SampleType (out of domain) */
} flacgen_config;

typedef struct flacgen_output {
    uint8_t *flac;           /* complete stream bytes */
    size_t flac_len;
    int32_t *pcm;            /* interleaved source PCM (unjustified), n_samples * channels */
    uint64_t pcm_len;
    uint64_t *frame_offsets; /* byte offset of each frame header */
    uint32_t n_frames;
    size_t frames_begin;     /* byte offset of the first frame */
    uint8_t md5[16];
} flacgen_output;

void flacgen_default_config(flacgen_config *c);
/* Returns 0 on success, a negative code if the requested configuration cannot be
 * written inside the parity domain (e.g. side channel overflow). */
int flacgen_generate(const flacgen_config *c, flacgen_output *out);
/* Same, but encodes the given interleaved PCM (n_samples = len / channels per channel,
 * unjustified values within bps) instead of the synthetic signal. */
int flacgen_generate_pcm(const flacgen_config *c, const int32_t *pcm, uint64_t len, flacgen_output *out);
void flacgen_free(flacgen_output *out);

#ifdef __cplusplus
}
#endif
#endif
