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

import org.apache.flink.runtime.causal.determinant.CorruptDeterminantArrayException;

import java.nio.ByteBuffer;
import java.util.NoSuchElementException;

public final class ClonosEngine implements AutoCloseable {

	static {
		System.loadLibrary("clonos_jni"); // links against libclonos_engine.so
	}

	public static final int CLG_OK = 0;
	public static final int CLG_E_INVALID_ARG = -1;
	public static final int CLG_E_CORRUPT_TAG = -2;
	public static final int CLG_E_TRUNCATED = -3;
	public static final int CLG_E_BAD_ENUM = -4;
	public static final int CLG_E_NEG_LEN = -5;
	public static final int CLG_E_BAD_SERIAL = -6;
	public static final int CLG_E_CONSUMER_BACKWARDS = -7;
	public static final int CLG_E_NO_CONSUMER = -8;
	public static final int CLG_E_GAP = -9;
	public static final int CLG_E_NOSPACE = -10;
	public static final int CLG_E_CAPACITY = -11;
	public static final int CLG_E_STATE = -12;
	public static final int CLG_E_DEVICE = -13;
	public static final int CLG_E_NO_LOG = -14;
	public static final int CLG_E_NOT_BUFFER_BUILT = -15;
	public static final int CLG_E_EPOCH_GAP = -16;
	// in-flight log types (InFlightLogConfig.java:44, taskmanager.inflight.type) and replay flags
	public static final int CLG_IFL_IN_MEMORY = 0;
	public static final int CLG_IFL_SPILLABLE = 1;
	public static final int CLG_IFL_CONTINUE = 1;
	public static final int CLG_IFL_NULL_ITERATOR = 1;
	public static final int CLG_IFL_REPLAYING = 2;

	/** The engine's default job (clg_config sharing depth). */
	public static final int DEFAULT_JOB = 0;

	private final long handle; // clg_engine*

	public ClonosEngine(int segmentBytes, int poolSegments, int device, int sharingDepth) {
		this(segmentBytes, poolSegments, device, sharingDepth, 0, 0);
	}

	/** inFlightSegmentBytes / inFlightPoolSegments: the in-flight log's own HBM pool (0: 32 KiB x 4096). */
	public ClonosEngine(int segmentBytes, int poolSegments, int device, int sharingDepth, int inFlightSegmentBytes,
						int inFlightPoolSegments) {
		long[] out = new long[1];
		check(nCreate(segmentBytes, poolSegments, device, sharingDepth, inFlightSegmentBytes, inFlightPoolSegments, out));
		this.handle = out[0];
	}

	public long handle() {
		return handle;
	}

	/** A JobCausalLog's scope on this engine (JobCausalLogFactory.java:56-67): JobID + its
	 *  ExecutionConfig.determinantSharingDepth.  Returns the job slot. */
	public int openJob(long jobIdLower, long jobIdUpper, int sharingDepth) {
		int[] out = new int[1];
		check(nJobOpen(handle, jobIdLower, jobIdUpper, sharingDepth, out));
		return out[0];
	}

	public void closeJob(int job) {
		check(nJobClose(handle, job));
	}

	/** CausalLogID fields (CausalLogID.java:38-60) of a log of `job` -> u32 log handle. */
	public int openLog(int job, short vertexId, boolean isMain, long irpLower, long irpUpper, byte subpartition) {
		int[] out = new int[1];
		check(nLogOpen(handle, job, vertexId, isMain, irpLower, irpUpper, subpartition, out));
		return out[0];
	}

	/** JobCausalLogImpl.notifyCheckpointComplete :230-246: the job's CAS + fan-out to its logs. */
	public boolean truncateAll(int job, long checkpointId) {
		int[] applied = new int[1];
		check(nTruncateAll(handle, job, checkpointId, applied));
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
		throw toException(status, nLastError());
	}

	/** The exception the reference throws at the point the status stands for. */
	public static RuntimeException toException(int status, String msg) {
		switch (status) {
			case CLG_E_CORRUPT_TAG: // SimpleDeterminantEncoder.decodeNext :92
				return new CorruptDeterminantArrayException(tagOf(msg));
			case CLG_E_BAD_ENUM: // ProcessingTimeCallbackID.Type.values()[ord] / CheckpointType.values()[ord]
				return new ArrayIndexOutOfBoundsException(msg);
			case CLG_E_NEG_LEN: // new byte[negative] (:235, :282)
				return new NegativeArraySizeException(msg);
			case CLG_E_TRUNCATED: // ByteBuf.readX past writerIndex
			case CLG_E_GAP: // ThreadCausalLogImpl.processUpstreamDelta: delta.readerIndex(< 0) (:143)
			case CLG_E_STATE: // makeDeltaUnsafe / getDeterminants index checks
				return new IndexOutOfBoundsException(msg);
			case CLG_E_CONSUMER_BACKWARDS: // ThreadCausalLogImpl.java:215-218
				return new RuntimeException("Consumer went backwards: " + msg);
			case CLG_E_NO_CONSUMER: // :245 / :256 dereference a missing ConsumerOffset
			case CLG_E_EPOCH_GAP: // ReplayIterator :133 / SpilledReplayIterator.EpochCursor (log.get(epoch) == null)
			case CLG_E_NO_LOG: // flatThreadCausalLogs.get(id) == null
				return new NullPointerException(msg);
			case CLG_E_NOT_BUFFER_BUILT: // ReplayingState.SubpartitionRecoveryThread :172-177
				return new RuntimeException("Subpartition has corrupt recovery buffer, expected buffer built: " + msg);
			case CLG_E_INVALID_ARG:
				return new IllegalArgumentException(msg);
			default: // CLG_E_NOSPACE (callers retry), CLG_E_CAPACITY (callers resize), CLG_E_DEVICE
				return new IllegalStateException("clonos engine status " + status + ": " + msg);
		}
	}

	/** The tag byte clg_last_error reports for CLG_E_CORRUPT_TAG ("... (tag N)"). */
	private static byte tagOf(String msg) {
		int i = msg.lastIndexOf("tag ");
		if (i < 0) {
			return 0;
		}
		int j = i + 4;
		while (j < msg.length() && (Character.isDigit(msg.charAt(j)) || msg.charAt(j) == '-')) {
			j++;
		}
		try {
			return (byte) Integer.parseInt(msg.substring(i + 4, j));
		} catch (NumberFormatException e) {
			return 0;
		}
	}

	/** In-flight iterator statuses (InMemorySubpartitionInFlightLogger.ReplayIterator): a skip past
	 *  the end is ListIterator.next()'s NoSuchElementException; a start epoch that is absent
	 *  (currentIterator == null) or a gap (logToReplay.get(++currentKey) == null) is a
	 *  NullPointerException.  clg_last_error names the case. */
	public static RuntimeException inFlightException(int status, String msg) {
		if (status == CLG_E_STATE && msg.contains("past the end")) {
			return new NoSuchElementException(msg);
		}
		if (status == CLG_E_STATE || status == CLG_E_EPOCH_GAP) {
			return new NullPointerException(msg);
		}
		return toException(status, msg);
	}

	// ---- natives (jni/clonos_jni.c) ------------------------------------------------------
	static native int nCreate(int segmentBytes, int poolSegments, int device, int sharingDepth, int iflSegmentBytes,
							  int iflPoolSegments, long[] out);
	static native void nDestroy(long engine);
	static native String nLastError();
	static native int nJobOpen(long engine, long jobIdLower, long jobIdUpper, int sharingDepth, int[] out);
	static native int nJobClose(long engine, int job);
	static native int nLogOpen(long engine, int job, short vertexId, boolean isMain, long irpLower, long irpUpper,
							   byte subpartition, int[] out);
	static native int nLogClose(long engine, int log);
	// in-flight (data) log, InMemorySubpartitionInFlightLogger (inflightlogging/, :28-207) or
	// SpillableSubpartitionInFlightLogger (:45-341): type CLG_IFL_IN_MEMORY / CLG_IFL_SPILLABLE
	static native int nIflOpen(long engine, int type, int[] out);
	static native int nIflClose(long engine, int ifl);
	static native int nIflLog(long engine, int ifl, long epoch, ByteBuffer direct, int off, int len);
	/** n buffers staged back to back in `direct` (lens[i] bytes, epoch epochs[i]), logged in order. */
	static native int nIflLogBatch(long engine, int ifl, long[] epochs, int[] lens, ByteBuffer direct, int n);
	static native int nIflNotifyCheckpointComplete(long engine, int ifl, long checkpointId);
	/** res = {status, n_buffers, remaining, len, total, total_buffers, end_epoch, flags}; sizes (i32)
	 *  and epochs (i64, native order) receive one entry per buffer.  maxBuffers (0: all) and
	 *  flags CLG_IFL_CONTINUE (take from the current iterator) apply to spillable logs only. */
	static native int nIflReplay(long engine, int ifl, long startEpoch, int ignoreBuffers, int maxBuffers, int flags,
		ByteBuffer out, ByteBuffer sizes, ByteBuffer epochs, long[] res);
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
	static native int nTruncateAll(long engine, int job, long checkpointId, int[] applied);

	// batched paths: LogReplayerImpl / ReplayingState decode, the piggyback serde, replay-prep
	static native int nDecodeLogs(long engine, int[] logs, long[] startEpochs, ByteBuffer off, ByteBuffer tag,
								  ByteBuffer v0, ByteBuffer wIdx, ByteBuffer wRc, ByteBuffer wV1, ByteBuffer wVarOff,
								  ByteBuffer wVarLen, ByteBuffer wSub, long[] result, long[] spanRecBase);
	/** clg_decode_logs_async: ctx[0] = a handle for nDecodeWait (the buffers stay reachable until then). */
	static native int nDecodeLogsAsync(long engine, int[] logs, long[] startEpochs, ByteBuffer off, ByteBuffer tag,
									   ByteBuffer v0, ByteBuffer wIdx, ByteBuffer wRc, ByteBuffer wV1, ByteBuffer wVarOff,
									   ByteBuffer wVarLen, ByteBuffer wSub, long[] ctx);
	/** clg_decode_wait: completes the decode nDecodeLogsAsync queued; result as nDecodeLogs. */
	static native int nDecodeWait(long engine, long ctx, long[] result, long[] spanRecBase);
	/** One span of host bytes decoded on the GPU (clg_decode_host); result as nDecodeLogs. */
	static native int nDecodeHost(long engine, ByteBuffer bytes, int off, int len, ByteBuffer recOff, ByteBuffer tag,
								  ByteBuffer v0, ByteBuffer wIdx, ByteBuffer wRc, ByteBuffer wV1, ByteBuffer wVarOff,
								  ByteBuffer wVarLen, ByteBuffer wSub, long[] result);
	/** out = {vertexId, isMain, irpLower, irpUpper, subpartition, job}. */
	static native int nLogGetId(long engine, int log, long[] out);
	static native int nEnrichBatch(long engine, int strategy, long[] requests, int[] logs, byte[] flags,
								   ByteBuffer out, long[] results, long[] total);
	static native int nProcessDelta(long engine, int job, int strategy, ByteBuffer msg, int off, int len,
									int[] handles, long[] result);
	static native int nReplayPrepare(long engine, short vertexId, ByteBuffer[] buffers, int[] lens, long[] subpartitions,
									 ByteBuffer off, ByteBuffer tag, ByteBuffer v0, ByteBuffer wIdx, ByteBuffer wRc,
									 ByteBuffer wV1, ByteBuffer wVarOff, ByteBuffer wVarLen, ByteBuffer wSub,
									 long[] result, ByteBuffer bufferSizes, long[] subpartitionResults);
}
