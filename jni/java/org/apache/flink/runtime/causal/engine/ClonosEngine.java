/*
 * ClonosEngine -- Java facade over libclonos_engine.so (include/clonos_engine.h) through
 * jni/clonos_jni.c.  One engine per TaskManager per GPU; it owns the HBM segment pool
 * that replaces the NetworkBufferPool-backed determinant buffers
 * (JobCausalLogFactory.java:56-67).  Every native method returns a status (0 = OK);
 * check() turns a non-zero status into the exception the reference throws at the same
 * point (see INTEGRATION.md, "Errors").
 *
 * Source-only: this container has no JDK, so the binding is not compiled here.
 */
package org.apache.flink.runtime.causal.engine;

import java.nio.ByteBuffer;

public final class ClonosEngine implements AutoCloseable {

	static {
		System.loadLibrary("clonos_jni"); // links against libclonos_engine.so
	}

	public static final int CLG_OK = 0;
	public static final int CLG_E_CORRUPT_TAG = -2;
	public static final int CLG_E_CONSUMER_BACKWARDS = -7;
	public static final int CLG_E_NO_CONSUMER = -8;
	public static final int CLG_E_NOSPACE = -10;
	public static final int CLG_E_CAPACITY = -11;
	public static final int CLG_E_STATE = -12;
	public static final int CLG_E_EPOCH_GAP = -16;

	private final long handle; // clg_engine*

	public ClonosEngine(int segmentBytes, int poolSegments, int device, int sharingDepth) {
		long[] out = new long[1];
		check(nCreate(segmentBytes, poolSegments, device, sharingDepth, out));
		this.handle = out[0];
	}

	public long handle() {
		return handle;
	}

	/** CausalLogID fields (CausalLogID.java:38-60) -> u32 log handle. */
	public int openLog(short vertexId, boolean isMain, long irpLower, long irpUpper, byte subpartition) {
		int[] out = new int[1];
		check(nLogOpen(handle, vertexId, isMain, irpLower, irpUpper, subpartition, out));
		return out[0];
	}

	/** JobCausalLogImpl.notifyCheckpointComplete :230-246 (CAS + fan-out). */
	public boolean truncateAll(long checkpointId) {
		int[] applied = new int[1];
		check(nTruncateAll(handle, checkpointId, applied));
		return applied[0] != 0;
	}

	@Override
	public void close() {
		nDestroy(handle);
	}

	public static void check(int status) {
		if (status == CLG_OK) {
			return;
		}
		String msg = nLastError();
		switch (status) {
			case CLG_E_CONSUMER_BACKWARDS:
				throw new RuntimeException("Consumer went backwards: " + msg); // ThreadCausalLogImpl.java:216
			case CLG_E_NO_CONSUMER:
				throw new NullPointerException(msg); // :245 / :256 dereference a missing ConsumerOffset
			case CLG_E_CORRUPT_TAG:
				throw new IllegalStateException("corrupt determinant array: " + msg);
			case CLG_E_EPOCH_GAP: // InMemorySubpartitionInFlightLogger.ReplayIterator :133
			case CLG_E_STATE:
				throw new NullPointerException(msg);
			default:
				throw new IllegalStateException("clonos engine status " + status + ": " + msg);
		}
	}

	// ---- natives (jni/clonos_jni.c) ------------------------------------------------------
	static native int nCreate(int segmentBytes, int poolSegments, int device, int sharingDepth, long[] out);
	static native void nDestroy(long engine);
	static native String nLastError();
	static native int nLogOpen(long engine, short vertexId, boolean isMain, long irpLower, long irpUpper,
							   byte subpartition, int[] out);
	static native int nLogClose(long engine, int log);
	// in-flight (data) log, InMemorySubpartitionInFlightLogger (inflightlogging/, :28-207)
	static native int nIflOpen(long engine, int[] out);
	static native int nIflClose(long engine, int ifl);
	static native int nIflLog(long engine, int ifl, long epoch, ByteBuffer direct, int off, int len);
	static native int nIflNotifyCheckpointComplete(long engine, int ifl, long checkpointId);
	/** res = {status, n_buffers, remaining, len, total, total_buffers, end_epoch}; sizes (i32) and
	 *  epochs (i64, native order) receive one entry per buffer. */
	static native int nIflReplay(long engine, int ifl, long startEpoch, int ignoreBuffers, ByteBuffer out,
		ByteBuffer sizes, ByteBuffer epochs, long[] res);
	/** bytes = direct buffer holding encoded records (SimpleDeterminantEncoder.encodeTo). */
	static native int nAppend(long engine, int log, long epoch, ByteBuffer direct, int off, int len);
	static native int nUpstreamDelta(long engine, int log, long epoch, int offsetFromEpoch, ByteBuffer direct,
									 int off, int len);
	static native int nLogLength(long engine, int log, int[] out);
	static native int nHasDelta(long engine, int log, long chLo, long chHi, long epoch, int[] out);
	static native int nOffsetFromEpoch(long engine, int log, long chLo, long chHi, int[] out);
	/** out[0] = bytes written, or the required size with CLG_E_CAPACITY. */
	static native int nGetDelta(long engine, int log, long chLo, long chHi, long epoch, ByteBuffer direct,
								int[] out);
	static native int nGetDeterminants(long engine, int log, long startEpoch, ByteBuffer direct, int[] out);
	static native int nNotifyCheckpointComplete(long engine, int log, long checkpointId);
	static native int nUnregisterConsumer(long engine, int log, long chLo, long chHi);
	static native int nTruncateAll(long engine, long checkpointId, int[] applied);

	// batched paths: LogReplayerImpl / ReplayingState decode, the piggyback serde, replay-prep
	static native int nDecodeLogs(long engine, int[] logs, long[] startEpochs, ByteBuffer off, ByteBuffer tag,
								  ByteBuffer v0, ByteBuffer wIdx, ByteBuffer wRc, ByteBuffer wV1, ByteBuffer wVarOff,
								  ByteBuffer wVarLen, ByteBuffer wSub, long[] result, long[] spanRecBase);
	static native int nEnrichBatch(long engine, int strategy, long[] requests, int[] logs, byte[] flags,
								   ByteBuffer out, long[] results, long[] total);
	static native int nProcessDelta(long engine, int strategy, ByteBuffer msg, int off, int len, int[] handles,
									long[] result);
	static native int nReplayPrepare(long engine, short vertexId, ByteBuffer mergedEvent, int len, long[] subpartitions,
									 ByteBuffer off, ByteBuffer tag, ByteBuffer v0, ByteBuffer wIdx, ByteBuffer wRc,
									 ByteBuffer wV1, ByteBuffer wVarOff, ByteBuffer wVarLen, ByteBuffer wSub,
									 long[] result, ByteBuffer bufferSizes, long[] subpartitionResults);
}
