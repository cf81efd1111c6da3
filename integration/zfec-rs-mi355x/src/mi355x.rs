//! Opt-in MI355X surface beyond the zfec-rs API (`zfec_rs::mi355x`).
//!
//! `piece.rs` reaches the GPU through `Fec::encode` / `Fec::decode` one chunk
//! at a time (crates/storb_base/src/piece.rs:328-329,383-386). The calls
//! below carry the speed-ups that per-chunk API cannot: a run of chunks in
//! one pipelined call with every piece id hashed on the GPU (the upload loop,
//! crates/storb_validator/src/upload.rs:418-420 encode + :623 blake3), the
//! download side's reconstructions batched (download.rs:453-465), async
//! single calls a tokio task can await instead of blocking a worker
//! (upload.rs:420, download.rs:464), and page-locked buffers the library
//! DMAs in place. INTEGRATION.md shows the call-site wiring.
//!
//! Every `extern "C"` here is checked against include/storb_rs.h by
//! tests/test_rust_binding.py (no Rust toolchain in the build image).
use std::marker::PhantomData;
use std::ops::{Deref, DerefMut};
use std::os::raw::{c_int, c_void};

use crate::{error, Error, StorbRsCtx};

#[repr(C)]
pub struct StorbRsOp {
    _private: [u8; 0],
}

extern "C" {
    fn storb_rs_ctx_create(device_ordinal: c_int, out: *mut *mut StorbRsCtx) -> c_int;
    fn storb_rs_ctx_destroy(ctx: *mut StorbRsCtx);
    fn storb_rs_block_size(k: u32, len: usize) -> usize;
    fn storb_rs_encode_chunks(
        ctx: *mut StorbRsCtx,
        k: u32,
        n: u32,
        data: *const u8,
        chunk_len: usize,
        nchunks: u32,
        parity_out: *mut u8,
    ) -> c_int;
    fn storb_rs_encode_chunks_hashed(
        ctx: *mut StorbRsCtx,
        k: u32,
        n: u32,
        data: *const u8,
        chunk_len: usize,
        nchunks: u32,
        parity_out: *mut u8,
        hashes_out: *mut u8,
    ) -> c_int;
    fn storb_rs_decode_chunks(
        ctx: *mut StorbRsCtx,
        k: u32,
        n: u32,
        block: usize,
        padlen: usize,
        nchunks: u32,
        shares: *const *const u8,
        share_idx: *const u32,
        nshares: *const u32,
        out: *mut u8,
        out_stride: usize,
    ) -> c_int;
    fn storb_rs_encode_async(
        ctx: *mut StorbRsCtx,
        k: u32,
        n: u32,
        data: *const u8,
        len: usize,
        parity_out: *const *mut u8,
        block_out: *mut usize,
        padlen_out: *mut usize,
        notify: Option<unsafe extern "C" fn(*mut c_void)>,
        user: *mut c_void,
        op: *mut *mut StorbRsOp,
    ) -> c_int;
    fn storb_rs_decode_async(
        ctx: *mut StorbRsCtx,
        k: u32,
        n: u32,
        shares: *const *const u8,
        share_idx: *const u32,
        nshares: u32,
        block: usize,
        padlen: usize,
        out: *mut u8,
        notify: Option<unsafe extern "C" fn(*mut c_void)>,
        user: *mut c_void,
        op: *mut *mut StorbRsOp,
    ) -> c_int;
    fn storb_rs_op_test(op: *const StorbRsOp) -> c_int;
    fn storb_rs_op_finish(op: *mut StorbRsOp) -> c_int;
    fn storb_rs_notify_fd(user: *mut c_void);
    fn storb_rs_host_alloc(len: usize, out: *mut *mut c_void) -> c_int;
    fn storb_rs_host_free(p: *mut c_void) -> c_int;
    fn storb_rs_host_register(p: *mut c_void, len: usize) -> c_int;
    fn storb_rs_host_unregister(p: *mut c_void) -> c_int;
    fn storb_blake3(data: *const u8, len: usize, out: *mut u8);
    fn storb_rs_device_numa_node(device: c_int) -> c_int;
    fn storb_rs_select_device(
        caller_node: c_int,
        device_nodes: *const c_int,
        ndev: c_int,
        ticket: u64,
    ) -> c_int;
}

// glibc, for the ops' wake-up descriptors (tokio AsyncFd / epoll).
extern "C" {
    fn eventfd(initval: u32, flags: c_int) -> c_int;
    fn close(fd: c_int) -> c_int;
}
const EFD_NONBLOCK: c_int = 0o4000;
const EFD_CLOEXEC: c_int = 0o2000000;
const EAGAIN: c_int = 6;

fn check(rc: c_int, ctx: *const StorbRsCtx) -> Result<(), Error> {
    if rc == 0 {
        Ok(())
    } else {
        Err(error(rc, ctx))
    }
}

/// blake3 of one shard: Storb's piece id (upload.rs:623, download.rs:158).
pub fn blake3(data: &[u8]) -> [u8; 32] {
    let mut out = [0u8; 32];
    unsafe { storb_blake3(data.as_ptr(), data.len(), out.as_mut_ptr()) };
    out
}

/// NUMA node of the host socket GPU `device` hangs off (None if unknown).
/// Per-chunk calls from a thread on another socket pay the socket link
/// ((4, 6) 1 MiB encode 59.5 vs 51.4 us): run the upload /
/// download workers on this node's CPUs (`/sys/devices/system/node/node<N>/cpulist`,
/// e.g. from a tokio runtime's `on_thread_start`).
pub fn device_numa_node(device: i32) -> Option<u32> {
    let n = unsafe { storb_rs_device_numa_node(device) };
    if n < 0 {
        None
    } else {
        Some(n as u32)
    }
}

/// The GPU `Context::new(-1)` gives the `ticket`-th context created by a
/// thread on NUMA node `caller_node` (None: node unknown), for a topology
/// given as each device's node: round-robin over the GPUs on the caller's
/// socket, over all GPUs when that socket has none. Pure; no device access.
pub fn select_device(caller_node: Option<u32>, device_nodes: &[i32], ticket: u64) -> Option<usize> {
    let node = caller_node.map(|n| n as c_int).unwrap_or(-1);
    let d = unsafe {
        storb_rs_select_device(node, device_nodes.as_ptr(), device_nodes.len() as c_int, ticket)
    };
    if d < 0 {
        None
    } else {
        Some(d as usize)
    }
}

/// A GPU context: streams, staging, table caches. Calls on one context are
/// serialised by the library; use one per thread for concurrency.
pub struct Context {
    ptr: *mut StorbRsCtx,
}
unsafe impl Send for Context {}
unsafe impl Sync for Context {}

impl Drop for Context {
    fn drop(&mut self) {
        unsafe { storb_rs_ctx_destroy(self.ptr) }
    }
}

/// The shares one chunk offers to a decode: (piece index, bytes). Any order;
/// the first k by index are used (decode_chunk, piece.rs:368-381).
pub type ChunkShares<'a> = Vec<(usize, &'a [u8])>;

impl Context {
    /// `device` >= 0 pins a GPU; -1 deals contexts round-robin over the node.
    pub fn new(device: i32) -> Result<Context, Error> {
        let mut p: *mut StorbRsCtx = std::ptr::null_mut();
        check(unsafe { storb_rs_ctx_create(device, &mut p) }, std::ptr::null())?;
        Ok(Context { ptr: p })
    }

    fn dims(k: usize, n: usize, chunk_len: usize, len: usize) -> Result<(usize, usize), Error> {
        if k == 0 || n < k || chunk_len == 0 || len % chunk_len != 0 {
            return Err(error(1, std::ptr::null()));
        }
        Ok((len / chunk_len, unsafe { storb_rs_block_size(k as u32, chunk_len) }))
    }

    /// Parity of a run of equal chunks laid end to end in `data` (the upload
    /// loop, upload.rs:418-420): chunk c's parity share p lands at
    /// `parity_out[(c * (n - k) + p) * B ..][.. B]`, B = ceil(chunk_len / k).
    pub fn encode_chunks(&self, k: usize, n: usize, data: &[u8], chunk_len: usize,
                         parity_out: &mut [u8]) -> Result<(), Error> {
        let (nch, b) = Self::dims(k, n, chunk_len, data.len())?;
        if parity_out.len() < nch * (n - k) * b {
            return Err(error(1, std::ptr::null()));
        }
        check(unsafe {
            storb_rs_encode_chunks(self.ptr, k as u32, n as u32, data.as_ptr(), chunk_len,
                                   nch as u32, parity_out.as_mut_ptr())
        }, self.ptr)
    }

    /// `encode_chunks` plus every share's piece id computed on the GPU:
    /// `hashes_out[c * n + i]` = blake3 of share i of chunk c (upload.rs:623).
    pub fn encode_chunks_hashed(&self, k: usize, n: usize, data: &[u8], chunk_len: usize,
                                parity_out: &mut [u8], hashes_out: &mut [[u8; 32]])
                                -> Result<(), Error> {
        let (nch, b) = Self::dims(k, n, chunk_len, data.len())?;
        if parity_out.len() < nch * (n - k) * b || hashes_out.len() < nch * n {
            return Err(error(1, std::ptr::null()));
        }
        check(unsafe {
            storb_rs_encode_chunks_hashed(self.ptr, k as u32, n as u32, data.as_ptr(), chunk_len,
                                          nch as u32, parity_out.as_mut_ptr(),
                                          hashes_out.as_mut_ptr() as *mut u8)
        }, self.ptr)
    }

    /// Reconstruct a batch of chunks of one (k, n, block, padlen) -- the
    /// download loop's reconstruct_chunk calls (download.rs:453-465) in one
    /// pipelined call. Chunk c's `k * block - padlen` bytes land at
    /// `out[c * out_stride ..]` (out_stride 0 = packed). Err(2) if a chunk
    /// has fewer than k distinct shares (reconstruct_chunk's Err).
    pub fn decode_chunks(&self, k: usize, n: usize, block: usize, padlen: usize,
                         chunks: &[ChunkShares<'_>], out: &mut [u8], out_stride: usize)
                         -> Result<(), Error> {
        let outlen = (k * block).checked_sub(padlen).ok_or_else(|| error(1, std::ptr::null()))?;
        let stride = if out_stride == 0 { outlen } else { out_stride };
        if chunks.is_empty() {
            return Ok(());
        }
        if stride < outlen || out.len() < (chunks.len() - 1) * stride + outlen {
            return Err(error(1, std::ptr::null()));
        }
        let mut ptrs = Vec::new();
        let mut idx = Vec::new();
        let mut cnt = Vec::with_capacity(chunks.len());
        for ch in chunks {
            cnt.push(ch.len() as u32);
            for (i, s) in ch {
                if s.len() < block {
                    return Err(error(1, std::ptr::null()));
                }
                ptrs.push(s.as_ptr());
                idx.push(*i as u32);
            }
        }
        check(unsafe {
            storb_rs_decode_chunks(self.ptr, k as u32, n as u32, block, padlen,
                                   chunks.len() as u32, ptrs.as_ptr(), idx.as_ptr(),
                                   cnt.as_ptr(), out.as_mut_ptr(), out_stride)
        }, self.ptr)
    }

    fn new_fd() -> Result<c_int, Error> {
        let fd = unsafe { eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC) };
        if fd < 0 {
            Err(error(4, std::ptr::null()))
        } else {
            Ok(fd)
        }
    }

    /// Start one chunk's encode (upload.rs:420) and return at once: the
    /// chunk is staged by the call, the parity is computed while the task
    /// does other work. `op.fd()` becomes readable when the device work is
    /// done (register it with tokio's AsyncFd); `op.finish()` returns the
    /// n - k parity shares.
    pub fn encode_async(&self, k: usize, n: usize, data: &[u8]) -> Result<EncodeOp<'_>, Error> {
        let b = if k == 0 { 0 } else { unsafe { storb_rs_block_size(k as u32, data.len()) } };
        let mut parity: Vec<Vec<u8>> = (k..n).map(|_| Vec::with_capacity(b.max(1))).collect();
        let ptrs: Vec<*mut u8> = parity.iter_mut().map(|v| v.as_mut_ptr()).collect();
        let fd = Self::new_fd()?;
        let (mut block, mut pad) = (0usize, 0usize);
        let mut op: *mut StorbRsOp = std::ptr::null_mut();
        let rc = unsafe {
            storb_rs_encode_async(self.ptr, k as u32, n as u32, data.as_ptr(), data.len(),
                                  ptrs.as_ptr(), &mut block, &mut pad, Some(storb_rs_notify_fd),
                                  fd as isize as *mut c_void, &mut op)
        };
        if rc != 0 {
            unsafe { close(fd) };
            return Err(error(rc, self.ptr));
        }
        Ok(EncodeOp { op, fd, parity, block, pad, _ctx: PhantomData })
    }

    /// Start one chunk's reconstruction (download.rs:464 -> decode_chunk):
    /// `op.finish()` returns its `k * block - padlen` bytes.
    pub fn decode_async(&self, k: usize, n: usize, shares: &[(usize, &[u8])], block: usize,
                        padlen: usize) -> Result<DecodeOp<'_>, Error> {
        let outlen = (k * block).checked_sub(padlen).ok_or_else(|| error(1, std::ptr::null()))?;
        let mut out: Vec<u8> = Vec::with_capacity(outlen.max(1));
        let ptrs: Vec<*const u8> = shares.iter().map(|(_, s)| s.as_ptr()).collect();
        let idx: Vec<u32> = shares.iter().map(|(i, _)| *i as u32).collect();
        if shares.iter().any(|(_, s)| s.len() < block) {
            return Err(error(1, std::ptr::null()));
        }
        let fd = Self::new_fd()?;
        let mut op: *mut StorbRsOp = std::ptr::null_mut();
        let rc = unsafe {
            storb_rs_decode_async(self.ptr, k as u32, n as u32, ptrs.as_ptr(), idx.as_ptr(),
                                  idx.len() as u32, block, padlen, out.as_mut_ptr(),
                                  Some(storb_rs_notify_fd), fd as isize as *mut c_void, &mut op)
        };
        if rc != 0 {
            unsafe { close(fd) };
            return Err(error(rc, self.ptr));
        }
        Ok(DecodeOp { op, fd, out, outlen, _ctx: PhantomData })
    }
}

/// An in-flight async encode. It borrows its context, so the context cannot
/// be destroyed under it; dropping it unfinished waits for the device work.
pub struct EncodeOp<'a> {
    op: *mut StorbRsOp,
    fd: c_int,
    parity: Vec<Vec<u8>>,
    block: usize,
    pad: usize,
    _ctx: PhantomData<&'a Context>,
}

/// An in-flight async decode (see `EncodeOp`).
pub struct DecodeOp<'a> {
    op: *mut StorbRsOp,
    fd: c_int,
    out: Vec<u8>,
    outlen: usize,
    _ctx: PhantomData<&'a Context>,
}

fn op_done(op: *mut StorbRsOp) -> Result<bool, Error> {
    match unsafe { storb_rs_op_test(op) } {
        0 => Ok(true),
        EAGAIN => Ok(false),
        rc => Err(error(rc, std::ptr::null())),
    }
}

impl<'a> EncodeOp<'a> {
    /// Readable (eventfd) once the device work is done.
    pub fn fd(&self) -> c_int {
        self.fd
    }
    pub fn is_done(&self) -> Result<bool, Error> {
        op_done(self.op)
    }
    /// (parity shares, padlen): waits if needed.
    pub fn finish(mut self) -> Result<(Vec<Vec<u8>>, usize), Error> {
        let rc = unsafe { storb_rs_op_finish(self.op) };
        self.op = std::ptr::null_mut();
        check(rc, std::ptr::null())?;
        let mut parity = std::mem::take(&mut self.parity);
        for v in parity.iter_mut() {
            unsafe { v.set_len(self.block) } // every byte written by the library
        }
        Ok((parity, self.pad))
    }
}

impl<'a> DecodeOp<'a> {
    pub fn fd(&self) -> c_int {
        self.fd
    }
    pub fn is_done(&self) -> Result<bool, Error> {
        op_done(self.op)
    }
    pub fn finish(mut self) -> Result<Vec<u8>, Error> {
        let rc = unsafe { storb_rs_op_finish(self.op) };
        self.op = std::ptr::null_mut();
        check(rc, std::ptr::null())?;
        let mut out = std::mem::take(&mut self.out);
        unsafe { out.set_len(self.outlen) } // every byte written by the library
        Ok(out)
    }
}

impl<'a> Drop for EncodeOp<'a> {
    fn drop(&mut self) {
        if !self.op.is_null() {
            unsafe { storb_rs_op_finish(self.op) }; // the outputs are still ours here
        }
        unsafe { close(self.fd) };
    }
}

impl<'a> Drop for DecodeOp<'a> {
    fn drop(&mut self) {
        if !self.op.is_null() {
            unsafe { storb_rs_op_finish(self.op) };
        }
        unsafe { close(self.fd) };
    }
}

/// Page-locked host memory from the library: chunk buffers the pipelined
/// calls DMA in place and the zero-copy kernels read over PCIe (upload.rs
/// :333-383 fills one chunk buffer at a time).
pub struct HostBuffer {
    ptr: *mut u8,
    len: usize,
}
unsafe impl Send for HostBuffer {}

impl HostBuffer {
    pub fn new(len: usize) -> Result<HostBuffer, Error> {
        let mut p: *mut c_void = std::ptr::null_mut();
        check(unsafe { storb_rs_host_alloc(len, &mut p) }, std::ptr::null())?;
        Ok(HostBuffer { ptr: p as *mut u8, len })
    }
}

impl Deref for HostBuffer {
    type Target = [u8];
    fn deref(&self) -> &[u8] {
        unsafe { std::slice::from_raw_parts(self.ptr, self.len) }
    }
}

impl DerefMut for HostBuffer {
    fn deref_mut(&mut self) -> &mut [u8] {
        unsafe { std::slice::from_raw_parts_mut(self.ptr, self.len) }
    }
}

impl Drop for HostBuffer {
    fn drop(&mut self) {
        unsafe { storb_rs_host_free(self.ptr as *mut c_void) }; // waits for the devices first
    }
}

/// A caller buffer made page-locked for as long as this lives (e.g. a
/// reused receive buffer on the download side).
pub struct Registration<'a> {
    ptr: *mut u8,
    _buf: PhantomData<&'a mut [u8]>,
}

pub fn register(buf: &mut [u8]) -> Result<Registration<'_>, Error> {
    check(unsafe { storb_rs_host_register(buf.as_mut_ptr() as *mut c_void, buf.len()) },
          std::ptr::null())?;
    Ok(Registration { ptr: buf.as_mut_ptr(), _buf: PhantomData })
}

impl<'a> Drop for Registration<'a> {
    fn drop(&mut self) {
        unsafe { storb_rs_host_unregister(self.ptr as *mut c_void) };
    }
}
