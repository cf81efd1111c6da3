//! `zfec-rs` API surface used by Storb, running on MI355X.
//!
//! Storb uses exactly: `Fec::new(k, m)`, `Fec::encode(&[u8])`,
//! `Fec::decode(&Vec<Chunk>, padding)`, `Chunk::new(data, index)` and the
//! field `Chunk.data` (crates/storb_base/src/piece.rs:9,328-329,375,383-386).
//! Each maps onto the C ABI of `include/storb_rs.h`. `m` is the TOTAL share
//! count, as in zfec. Errors are `Err(Error)`, which Storb `.expect()`s.
//!
//! NOTE: no Rust toolchain exists in the build image of this project, so
//! this crate is written against the header but has not been compiled here;
//! the same boundary is exercised from C++ (tests/cpp/test_piece.cpp) and
//! Python ctypes (tests/).
use std::cell::RefCell;
use std::ffi::CStr;
use std::fmt;
use std::os::raw::{c_char, c_int};

/// Batched, hashed, async and page-locked calls beyond the zfec-rs API.
pub mod mi355x;

#[repr(C)]
pub struct StorbRsCtx {
    _private: [u8; 0],
}

extern "C" {
    fn storb_rs_ctx_create(device_ordinal: c_int, out: *mut *mut StorbRsCtx) -> c_int;
    fn storb_rs_ctx_destroy(ctx: *mut StorbRsCtx);
    fn storb_rs_strerror(code: c_int) -> *const c_char;
    fn storb_rs_last_error(ctx: *const StorbRsCtx) -> *const c_char;
    fn storb_rs_check_params(k: u32, n: u32) -> c_int;
    fn storb_rs_block_size(k: u32, len: usize) -> usize;
    fn storb_rs_encode_shares(
        ctx: *mut StorbRsCtx,
        k: u32,
        n: u32,
        data: *const u8,
        len: usize,
        shares_out: *const *mut u8,
        block_out: *mut usize,
        padlen_out: *mut usize,
    ) -> c_int;
    fn storb_rs_decode(
        ctx: *mut StorbRsCtx,
        k: u32,
        n: u32,
        shares: *const *const u8,
        share_idx: *const u32,
        nshares: u32,
        block: usize,
        padlen: usize,
        out: *mut u8,
    ) -> c_int;
}

/// Error returned by the MI355X codec (code from `storb_rs.h`).
#[derive(Clone, PartialEq, Eq)]
pub struct Error {
    pub code: i32,
    pub message: String,
}

impl fmt::Debug for Error {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        write!(f, "zfec-rs(mi355x) error {}: {}", self.code, self.message)
    }
}
impl fmt::Display for Error {
    fn fmt(&self, f: &mut fmt::Formatter<'_>) -> fmt::Result {
        fmt::Debug::fmt(self, f)
    }
}
impl std::error::Error for Error {}

fn error(code: c_int, ctx: *const StorbRsCtx) -> Error {
    let mut message = unsafe { CStr::from_ptr(storb_rs_strerror(code)) }
        .to_string_lossy()
        .into_owned();
    if !ctx.is_null() {
        let d = unsafe { CStr::from_ptr(storb_rs_last_error(ctx)) }.to_string_lossy();
        if !d.is_empty() {
            message.push_str(": ");
            message.push_str(&d);
        }
    }
    Error { code, message }
}

/// One context per calling thread (tokio workers are long-lived); its GPU
/// is chosen round-robin, so concurrent uploads spread over the node.
struct Ctx(*mut StorbRsCtx);
impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { storb_rs_ctx_destroy(self.0) }
    }
}
thread_local! {
    static CTX: RefCell<Option<Ctx>> = RefCell::new(None);
}

fn with_ctx<T>(f: impl FnOnce(*mut StorbRsCtx) -> Result<T, Error>) -> Result<T, Error> {
    CTX.with(|cell| {
        let mut slot = cell.borrow_mut();
        if slot.is_none() {
            let mut p: *mut StorbRsCtx = std::ptr::null_mut();
            let rc = unsafe { storb_rs_ctx_create(-1, &mut p) };
            if rc != 0 {
                return Err(error(rc, std::ptr::null()));
            }
            *slot = Some(Ctx(p));
        }
        f(slot.as_ref().unwrap().0)
    })
}

/// A share: `data` plus its index (0..k data, k..m parity).
#[derive(Debug, Clone, PartialEq, Eq)]
pub struct Chunk {
    pub data: Vec<u8>,
    pub index: usize,
}

impl Chunk {
    pub fn new(data: Vec<u8>, index: usize) -> Self {
        Chunk { data, index }
    }
}

/// Systematic Vandermonde RS code over GF(2^8) (zfec's fec.c construction).
#[derive(Debug, Clone)]
pub struct Fec {
    k: usize,
    m: usize,
}

impl Fec {
    pub fn new(k: usize, m: usize) -> Result<Fec, Error> {
        if k > 256 || m > 256 || unsafe { storb_rs_check_params(k as u32, m as u32) } != 0 {
            return Err(error(1, std::ptr::null()));
        }
        Ok(Fec { k, m })
    }

    /// All `m` shares in index order and the zero-padding length. One call
    /// writes every share: the library copies the k data shares (the last
    /// one zero-padded) on its host pool while the kernel computes parity,
    /// so the shim neither zero-fills nor copies anything itself.
    pub fn encode(&self, data: &[u8]) -> Result<(Vec<Chunk>, usize), Error> {
        let (k, m) = (self.k, self.m);
        let b = unsafe { storb_rs_block_size(k as u32, data.len()) };
        let mut bufs: Vec<Vec<u8>> = (0..m).map(|_| Vec::with_capacity(b.max(1))).collect();
        let ptrs: Vec<*mut u8> = bufs.iter_mut().map(|v| v.as_mut_ptr()).collect();
        let (mut block, mut pad) = (0usize, 0usize);
        with_ctx(|ctx| {
            let rc = unsafe {
                storb_rs_encode_shares(ctx, k as u32, m as u32, data.as_ptr(), data.len(),
                                       ptrs.as_ptr(), &mut block, &mut pad)
            };
            if rc != 0 { Err(error(rc, ctx)) } else { Ok(()) }
        })?;
        let chunks = bufs
            .into_iter()
            .enumerate()
            .map(|(i, mut v)| {
                unsafe { v.set_len(b) } // all b bytes written by storb_rs_encode_shares
                Chunk::new(v, i)
            })
            .collect();
        Ok((chunks, pad))
    }

    /// The original bytes from >= k shares (first k by index are used).
    pub fn decode(&self, encoded_data: &Vec<Chunk>, padding: usize) -> Result<Vec<u8>, Error> {
        let k = self.k;
        if encoded_data.len() < k {
            return Err(error(2, std::ptr::null()));
        }
        let b = encoded_data[0].data.len();
        if b == 0 || padding >= k * b || encoded_data.iter().any(|c| c.data.len() != b) {
            return Err(error(1, std::ptr::null()));
        }
        let ptrs: Vec<*const u8> = encoded_data.iter().map(|c| c.data.as_ptr()).collect();
        let idx: Vec<u32> = encoded_data.iter().map(|c| c.index as u32).collect();
        let outlen = k * b - padding;
        let mut out: Vec<u8> = Vec::with_capacity(outlen);
        with_ctx(|ctx| {
            let rc = unsafe {
                storb_rs_decode(ctx, k as u32, self.m as u32, ptrs.as_ptr(), idx.as_ptr(),
                                idx.len() as u32, b, padding, out.as_mut_ptr())
            };
            if rc != 0 { Err(error(rc, ctx)) } else { Ok(()) }
        })?;
        unsafe { out.set_len(outlen) } // every byte written by storb_rs_decode
        Ok(out)
    }
}
