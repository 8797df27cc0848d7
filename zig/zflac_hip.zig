//! zflac_hip.zig -- drop-in `decode` for Senryoku/zflac backed by libzflac_hip.so (MI355X).
//!
//! What a zflac maintainer adds as `src/zflac_hip.zig` (INTEGRATION.md has the build.zig
//! lines). Same signature and result type as the reference entry point
//!
//!     pub fn decode(allocator: std.mem.Allocator, reader: anytype) !DecodedFLAC  // src/zflac.zig:216-217
//!
//! and the same ownership contract: the samples live in `_samples_backing`, allocated from
//! the caller's allocator with 32-byte alignment (src/zflac.zig:331) and freed by
//! `DecodedFLAC.deinit(allocator)` (src/zflac.zig:25-27).
//!
//! The C side is include/zflac_hip.h (two-phase: open -> caller allocation -> read). This
//! file is not compiled in this repository (the build image has no `zig`); its C twin,
//! tests/c/abi_consumer.c, binds the same header with the same error mapping, the same
//! struct-layout assertions and the same 32-byte aligned caller allocation, and runs in the
//! GPU test suite (tests/test_c_consumer.py).
const std = @import("std");
const zflac = @import("zflac.zig");
const c = @cImport(@cInclude("zflac_hip.h"));

// zflac_info / zflac_stream as a Zig `extern struct` lays them out: the same offsets the C
// consumer static_asserts (tests/c/abi_consumer.c), so both sides bind one layout.
comptime {
    std.debug.assert(@sizeOf(c.zflac_info) == 24);
    std.debug.assert(@offsetOf(c.zflac_info, "channels") == 0);
    std.debug.assert(@offsetOf(c.zflac_info, "bits_per_sample") == 1);
    std.debug.assert(@offsetOf(c.zflac_info, "sample_kind") == 2);
    std.debug.assert(@offsetOf(c.zflac_info, "sample_rate") == 4);
    std.debug.assert(@offsetOf(c.zflac_info, "n_samples") == 8);
    std.debug.assert(@offsetOf(c.zflac_info, "samples_bytes") == 16);
    std.debug.assert(@sizeOf(c.zflac_stream) == 2 * @sizeOf(usize));
}

/// zflac's error set (src/zflac.zig; SURVEY.md App. A.3) plus the device-side extras.
pub const Error = error{
    InvalidSignature, // src/zflac.zig:220
    InvalidMetadataHeader, // :248
    MissingStreaminfo, // :309
    Unimplemented, // :263
    InvalidChecksum, // :280
    InvalidFrameHeader, // :352,357,361,372,405
    InconsistentParameters, // :386,391
    InvalidCodedNumber, // :206
    InvalidSubframeHeader, // :431,471,542
    InvalidResidualCodingMethod, // :618
    EndOfStream, // std.io reader
    OutOfMemory, // allocator
    DeviceError, // no GPU / HIP failure (no zflac equivalent)
    InvalidArgument, // bad handle or buffer size (a shim bug)
    OutOfDomain, // an input on which Debug zflac traps (SURVEY.md App. A)
    FrameCrcMismatch, // only with decodeWithFlags(.., c.ZFLAC_FLAG_CHECK_CRC16)
};

/// One case per ZFLAC_E_* code. tests/c/abi_consumer.c `shim_error_name` is the same switch,
/// checked against zflac_hip_error_name() for every code.
pub fn check(rc: c_int) Error!void {
    return switch (rc) {
        c.ZFLAC_OK => {},
        c.ZFLAC_E_INVALID_SIGNATURE => error.InvalidSignature,
        c.ZFLAC_E_INVALID_METADATA_HEADER => error.InvalidMetadataHeader,
        c.ZFLAC_E_MISSING_STREAMINFO => error.MissingStreaminfo,
        c.ZFLAC_E_UNIMPLEMENTED => error.Unimplemented,
        c.ZFLAC_E_INVALID_CHECKSUM => error.InvalidChecksum,
        c.ZFLAC_E_INVALID_FRAME_HEADER => error.InvalidFrameHeader,
        c.ZFLAC_E_INCONSISTENT_PARAMETERS => error.InconsistentParameters,
        c.ZFLAC_E_INVALID_CODED_NUMBER => error.InvalidCodedNumber,
        c.ZFLAC_E_INVALID_SUBFRAME_HEADER => error.InvalidSubframeHeader,
        c.ZFLAC_E_INVALID_RESIDUAL_CODING => error.InvalidResidualCodingMethod,
        c.ZFLAC_E_END_OF_STREAM => error.EndOfStream,
        c.ZFLAC_E_OUT_OF_MEMORY => error.OutOfMemory,
        c.ZFLAC_E_DEVICE => error.DeviceError,
        c.ZFLAC_E_INVALID_ARGUMENT => error.InvalidArgument,
        c.ZFLAC_E_OUT_OF_DOMAIN => error.OutOfDomain,
        c.ZFLAC_E_FRAME_CRC => error.FrameCrcMismatch,
        else => error.DeviceError,
    };
}

/// Same contract as zflac.decode (src/zflac.zig:216): caller owns the returned memory.
pub fn decode(allocator: std.mem.Allocator, reader: anytype) !zflac.DecodedFLAC {
    return decodeWithFlags(allocator, reader, 0);
}

/// decode() with zflac_hip_open_ex flags (c.ZFLAC_FLAG_CHECK_CRC16: frame CRC-16 checked on
/// the device, which zflac itself skips at src/zflac.zig:548-551).
pub fn decodeWithFlags(allocator: std.mem.Allocator, reader: anytype, flags: c_int) !zflac.DecodedFLAC {
    // zflac reads the stream once and never seeks; the device needs the whole stream.
    const bytes = try reader.readAllAlloc(allocator, std.math.maxInt(usize));
    defer allocator.free(bytes);

    var info: c.zflac_info = undefined;
    var h: ?*c.zflac_batch = null;
    const rc = c.zflac_hip_open_ex(bytes.ptr, bytes.len, 0, flags, &h, &info);
    defer if (h) |p| c.zflac_hip_close(p);
    try check(rc);

    // src/zflac.zig:331: the backing comes from the caller's allocator, 32-byte aligned
    const samples_backing = try allocator.allocWithOptions(u8, @intCast(info.samples_bytes), 32, null);
    errdefer allocator.free(samples_backing);
    try check(c.zflac_hip_read(h, samples_backing.ptr, samples_backing.len)); // MD5 -> InvalidChecksum (:279-280)

    const n: usize = @intCast(info.n_samples);
    // Each arm casts through [*]align(32) T exactly as src/zflac.zig:334 does, so the slice is
    // []align(32) T and coerces to the `Samples` union's arms (src/zflac.zig:12-16).
    return .{
        .channels = info.channels,
        .sample_rate = @intCast(info.sample_rate),
        .bits_per_sample = info.bits_per_sample,
        .samples = switch (info.sample_kind) {
            c.ZFLAC_S8 => .{ .s8 = @as([*]align(32) i8, @alignCast(@ptrCast(samples_backing.ptr)))[0..n] },
            c.ZFLAC_S16 => .{ .s16 = @as([*]align(32) i16, @alignCast(@ptrCast(samples_backing.ptr)))[0..n] },
            c.ZFLAC_S32 => .{ .s32 = @as([*]align(32) i32, @alignCast(@ptrCast(samples_backing.ptr)))[0..n] },
            else => return error.DeviceError,
        },
        ._samples_backing = samples_backing,
    };
}

test "zflac_hip decodes RFC 9639 example 3 (tests/basic.zig:77-95)" {
    // the stream and the expected PCM of tests/basic.zig:77-95 (tests/golden/basic_kat.json)
    const data = [_]u8{
        0x66, 0x4c, 0x61, 0x43, 0x80, 0x00, 0x00, 0x22, 0x10, 0x00, 0x10, 0x00, 0x00, 0x00, 0x1f, 0x00,
        0x00, 0x1f, 0x07, 0xd0, 0x00, 0x70, 0x00, 0x00, 0x00, 0x18, 0xf8, 0xf9, 0xe3, 0x96, 0xf5, 0xcb,
        0xcf, 0xc6, 0xdc, 0x80, 0x7f, 0x99, 0x77, 0x90, 0x6b, 0x32, 0xff, 0xf8, 0x68, 0x02, 0x00, 0x17,
        0xe9, 0x44, 0x00, 0x4f, 0x6f, 0x31, 0x3d, 0x10, 0x47, 0xd2, 0x27, 0xcb, 0x6d, 0x09, 0x08, 0x31,
        0x45, 0x2b, 0xdc, 0x28, 0x22, 0x22, 0x80, 0x57, 0xa3,
    };
    const expected = [_]i8{ 0, 79, 111, 78, 8, -61, -90, -68, -13, 42, 67, 53, 13, -27, -46, -38, -12, 14, 24, 19, 6, -4, -5, 0 };
    var fbs = std.io.fixedBufferStream(&data);
    const d = try decode(std.testing.allocator, fbs.reader());
    defer d.deinit(std.testing.allocator);
    try std.testing.expectEqual(@as(u8, 1), d.channels);
    try std.testing.expectEqualSlices(i8, &expected, d.samples.s8);
}
