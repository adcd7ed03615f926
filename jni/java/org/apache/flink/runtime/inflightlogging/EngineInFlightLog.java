/*
 * InFlightLog over the MI355X engine (C-ABI clg_ifl_*, jni/clonos_jni.c): a drop-in for
 * InMemorySubpartitionInFlightLogger (InMemorySubpartitionInFlightLogger.java:28-207) and for
 * the default SpillableSubpartitionInFlightLogger (SpillableSubpartitionInFlightLogger.java:45-341,
 * InFlightLogConfig.java:44), by type.  Buffer bytes are copied into HBM on log() and the Java
 * Buffer is recycled at once; a replay gathers buffers from HBM in GPU calls and hands them out
 * as Buffers taken from the in-flight buffer pool.  In-memory: one call drains the whole
 * iterator.  Spillable: the iterator is live (SpilledReplayIterator.notifyNewBufferAdded :262):
 * it takes REPLAY_CHUNK buffers per call and continues the engine's current iterator, so buffers
 * logged during the replay reach it.  Wiring: InMemoryInFlightLogFactory returns
 * `new EngineInFlightLog(engine, CLG_IFL_IN_MEMORY)` and SpillableInFlightLogFactory
 * `new EngineInFlightLog(engine, CLG_IFL_SPILLABLE)` (INTEGRATION.md).
 */
package org.apache.flink.runtime.inflightlogging;

import org.apache.flink.runtime.causal.engine.ClonosEngine;
import org.apache.flink.runtime.io.network.buffer.Buffer;
import org.apache.flink.runtime.io.network.buffer.BufferPool;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;

import static org.apache.flink.runtime.causal.engine.ClonosEngine.*;

public class EngineInFlightLog implements InFlightLog {

	private final ClonosEngine engine;
	private final int ifl;
	private final int type;
	private BufferPool inFlightBufferPool;
	private static final int REPLAY_CHUNK = 64; // spillable: buffers taken per engine call

	// log() stages buffers host-side and hands them to the engine in batches (one upload and
	// one scatter kernel per batch instead of a GPU round trip per network buffer); every other
	// operation flushes first, so the engine always sees the buffers in log() order
	private static final int STAGE_BYTES = 1 << 20;
	private static final int STAGE_BUFFERS = 256;
	private final ByteBuffer stage = ByteBuffer.allocateDirect(STAGE_BYTES);
	private final long[] stagedEpochs = new long[STAGE_BUFFERS];
	private final int[] stagedLens = new int[STAGE_BUFFERS];
	private int staged;
	// a batch is being handed to the engine (the staged arrays, or one large buffer): it may
	// wait for pool space (backpressure, wait() releases the monitor), and meanwhile no other
	// thread touches the stage or submits, so buffers reach the engine once and in log() order
	private boolean submitting;
	private boolean closed;
	// a checkpoint completed while a batch waited for pool space: truncated right after the
	// batch is accepted (Long.MIN_VALUE: none), so the notifier never waits for the batch
	private long pendingTruncation = Long.MIN_VALUE;
	// that truncation's failure, kept apart from the batch's append status: the caller clears
	// an accepted batch first (the engine holds its buffers), then raises it (CLG_OK: none)
	private int truncationStatus = CLG_OK;

	public EngineInFlightLog(ClonosEngine engine) {
		this(engine, CLG_IFL_IN_MEMORY);
	}

	public EngineInFlightLog(ClonosEngine engine, int type) {
		this.engine = engine;
		this.type = type;
		int[] h = new int[1];
		check(nIflOpen(engine.handle(), type, h));
		this.ifl = h[0];
	}

	@Override
	public void registerBufferPool(BufferPool bufferPool) {
		this.inFlightBufferPool = bufferPool;
	}

	@Override
	public synchronized void log(Buffer buffer, long epochID, boolean isFinished) { // :44-48
		awaitNoSubmit();
		ByteBuffer nio = buffer.getNioBufferReadable();
		int n = nio.remaining();
		if (n > stage.remaining() || staged == STAGE_BUFFERS) {
			flush();
		}
		if (n > STAGE_BYTES) { // larger than the stage: a batch of its own
			ByteBuffer direct = nio.isDirect() ? nio.slice() : ByteBuffer.allocateDirect(n).put(nio.duplicate());
			check(submit(new long[]{epochID}, new int[]{n}, direct, 1));
			raiseTruncation();
			return;
		}
		stage.put(nio.duplicate());
		stagedEpochs[staged] = epochID;
		stagedLens[staged] = n;
		staged++;
	}

	private void flush() {
		awaitNoSubmit();
		if (staged == 0) {
			return;
		}
		int st = submit(stagedEpochs, stagedLens, stage, staged);
		if (accepted(st)) { // logged (CLG_E_STATE too: every buffer was appended first), so never again
			stage.clear();
			staged = 0;
		}
		check(st);
		raiseTruncation();
	}

	/** A deferred truncation that failed in submit(): raised once its batch is cleared. */
	private void raiseTruncation() {
		int t = truncationStatus;
		truncationStatus = CLG_OK;
		check(t);
	}

	/** The engine appended the batch: CLG_OK, or CLG_E_STATE (spillable log() while replaying
	 *  without an iterator, :98-99, after the buffers were appended). */
	private static boolean accepted(int st) {
		return st == CLG_OK || st == CLG_E_STATE;
	}

	private void awaitNoSubmit() {
		while (submitting) {
			waitQuietly();
		}
	}

	private void waitQuietly() {
		try {
			wait(10);
		} catch (InterruptedException e) {
			Thread.currentThread().interrupt();
			throw new RuntimeException(e);
		}
	}

	// Backpressure: a full in-flight pool (CLG_E_NOSPACE, nothing logged) waits until a
	// checkpoint completes and frees epochs (notifyCheckpointComplete wakes us), then retries.
	// Every in-flight log of the engine shares one pool, and the reference notifies the
	// subpartitions one after another on one thread (EpochTrackerImpl.java:140-142), so the
	// notifier must not wait for this batch: the truncation it records is applied here, once
	// the batch is accepted.
	// The batch's arrays and bytes are the live stage while it waits (wait() releases the
	// monitor): nothing else touches them until it returns (log() and flush() wait for the
	// submit, notifyCheckpointComplete leaves the stage to pendingTruncation).  Returns the
	// append's status alone; the caller clears what was accepted, then raises it and then a
	// failed deferred truncation (truncationStatus; the truncation stays pending, so the next
	// accepted batch applies it again).
	private int submit(long[] epochs, int[] lens, ByteBuffer bytes, int n) {
		submitting = true;
		try {
			int st;
			while ((st = nIflLogBatch(engine.handle(), ifl, epochs, lens, bytes, n)) == CLG_E_NOSPACE) {
				if (closed) {
					throw new IllegalStateException("in-flight log closed while waiting for pool space");
				}
				waitQuietly();
			}
			long cp = pendingTruncation;
			if (cp != Long.MIN_VALUE && accepted(st)) {
				// the batch was logged before the notification: its epochs below cp go too
				int tst = nIflNotifyCheckpointComplete(engine.handle(), ifl, cp);
				if (tst == CLG_OK) {
					pendingTruncation = Long.MIN_VALUE;
				} else {
					truncationStatus = tst;
				}
			}
			return st; // CLG_E_STATE: spillable log() while replaying without an iterator (:98-99, NPE)
		} finally {
			submitting = false;
			notifyAll();
		}
	}

	@Override
	public synchronized void notifyCheckpointComplete(long checkpointId) { // in-memory :51-70, spillable :106-123
		// free the pool first: a log() waiting for space (backpressure) can then finish
		check(nIflNotifyCheckpointComplete(engine.handle(), ifl, checkpointId));
		notifyAll();
		// staged buffers of truncated epochs never reach HBM; a batch waiting for space right now
		// is truncated by submit() once it is accepted (the reference truncates every buffer
		// logged before the notification).  While a batch is submitted the stage IS that batch
		// (or empty: a large buffer goes alone after a flush), and submit() still reads its
		// arrays and bytes, so it is left alone: pendingTruncation covers it
		if (submitting) {
			pendingTruncation = Math.max(pendingTruncation, checkpointId);
		} else {
			dropStagedBelow(checkpointId);
		}
	}

	private void dropStagedBelow(long checkpointId) {
		int keep = 0, rd = 0, wr = 0;
		for (int i = 0; i < staged; i++) {
			int n = stagedLens[i];
			if (stagedEpochs[i] >= checkpointId) {
				if (rd != wr) {
					byte[] tmp = new byte[n];
					ByteBuffer src = stage.duplicate();
					src.position(rd).limit(rd + n);
					src.get(tmp);
					ByteBuffer dst = stage.duplicate();
					dst.position(wr);
					dst.put(tmp);
				}
				stagedEpochs[keep] = stagedEpochs[i];
				stagedLens[keep] = n;
				keep++;
				wr += n;
			}
			rd += n;
		}
		staged = keep;
		stage.position(wr);
	}

	@Override
	public synchronized InFlightLogIterator<Buffer> getInFlightIterator(long startEpochID, int ignoreBuffers) {
		flush();
		if (type == CLG_IFL_SPILLABLE) { // :126-142
			Chunk c = fetch(startEpochID, ignoreBuffers, 0);
			if ((c.flags & CLG_IFL_NULL_ITERATOR) != 0) {
				return null; // tailMap(epochID) is empty
			}
			return new LiveReplay(c);
		}
		Chunk c = fetch(startEpochID, ignoreBuffers, 0);
		return new Replay(c);
	}

	/** One engine call: a new iterator (flags 0) or the next buffers of the current one
	 *  (CLG_IFL_CONTINUE), sized first, then gathered into direct buffers. */
	private Chunk fetch(long startEpochID, int ignoreBuffers, int flags) {
		int max = type == CLG_IFL_SPILLABLE ? REPLAY_CHUNK : 0;
		long[] res = new long[8];
		int st = nIflReplay(engine.handle(), ifl, startEpochID, ignoreBuffers, max, flags, null, null, null, res);
		if (st != CLG_OK && st != CLG_E_CAPACITY) {
			check(st);
		}
		ByteBuffer out = ByteBuffer.allocateDirect((int) Math.max(1, res[4]));
		ByteBuffer sizes = ByteBuffer.allocateDirect((int) Math.max(4, 4 * res[5])).order(ByteOrder.nativeOrder());
		ByteBuffer epochs = ByteBuffer.allocateDirect((int) Math.max(8, 8 * res[5])).order(ByteOrder.nativeOrder());
		check(nIflReplay(engine.handle(), ifl, startEpochID, ignoreBuffers, max, flags, out, sizes, epochs, res));
		int status = (int) res[0];
		if (status != CLG_OK && status != CLG_E_EPOCH_GAP) { // the skip inside getInFlightIterator threw
			throw inFlightException(status, nLastError());
		}
		return new Chunk(out, sizes, epochs, (int) res[1], (int) res[2], res[6], status, (int) res[7]);
	}

	/** Buffers of one engine call. */
	private static final class Chunk {
		final ByteBuffer bytes;
		final ByteBuffer sizes;
		final ByteBuffer epochs;
		final int count;
		final int remaining; // numberRemaining() before these buffers were taken
		final long endEpoch;
		final int status;
		final int flags;
		int next;
		int pos;

		Chunk(ByteBuffer bytes, ByteBuffer sizes, ByteBuffer epochs, int count, int remaining, long endEpoch,
			int status, int flags) {
			this.bytes = bytes;
			this.sizes = sizes;
			this.epochs = epochs;
			this.count = count;
			this.remaining = remaining;
			this.endEpoch = endEpoch;
			this.status = status;
			this.flags = flags;
		}

		boolean has() {
			return next < count;
		}

		long epoch() {
			return next < count ? epochs.getLong(8 * next) : endEpoch;
		}
	}

	private Buffer materialise(Chunk c, boolean advance) {
		int n = c.sizes.getInt(4 * c.next);
		Buffer b;
		try {
			b = inFlightBufferPool.requestBufferBlocking();
		} catch (IOException | InterruptedException e) {
			throw new RuntimeException(e);
		}
		ByteBuffer src = c.bytes.duplicate();
		src.position(c.pos).limit(c.pos + n);
		b.getMemorySegment().put(0, src, n);
		b.setSize(n);
		if (advance) {
			c.pos += n;
			c.next++;
		}
		return b;
	}

	@Override
	public void destroyBufferPools() {
	}

	@Override
	public synchronized void close() { // :90-94
		closed = true;
		notifyAll();
		awaitNoSubmit();
		staged = 0;
		stage.clear();
		check(nIflClose(engine.handle(), ifl));
	}

	@Override
	public BufferPool getInFlightBufferPool() {
		return inFlightBufferPool;
	}

	/** The drained in-memory ReplayIterator (:107-201): buffers materialised from the gathered bytes. */
	private final class Replay extends InFlightLogIterator<Buffer> {
		private final Chunk c;
		private int left;

		Replay(Chunk c) {
			this.c = c;
			this.left = c.remaining;
		}

		@Override
		public boolean hasNext() {
			// at a gap the reference still sees the last buffer before it (:146-149); next() throws (:156 -> :133)
			return c.has() || c.status == CLG_E_EPOCH_GAP;
		}

		@Override
		public Buffer next() {
			if (!c.has()) {
				check(c.status); // CLG_E_EPOCH_GAP -> the reference's NullPointerException
				throw new java.util.NoSuchElementException();
			}
			left--;
			return materialise(c, true);
		}

		@Override
		public Buffer peekNext() {
			if (!c.has()) {
				throw new java.util.NoSuchElementException();
			}
			return materialise(c, false);
		}

		@Override
		public int numberRemaining() {
			return left;
		}

		/** ReplayIterator.getEpoch (:181-183): currentKey, i.e. the epoch of the buffer the next
		 *  next() returns -- PipelinedSubpartition.getReplayedBufferUnsafe (:306-320) stamps it on
		 *  the BufferAndBacklog -- and, once drained, the epoch the iterator stopped in. */
		@Override
		public long getEpoch() {
			return c.epoch();
		}

		@Override
		public void close() {
			c.next = c.count;
		}
	}

	/** The spillable logger's live SpilledReplayIterator (:60-401): REPLAY_CHUNK buffers per engine
	 *  call; an exhausted chunk continues the engine's current iterator, which also holds the
	 *  buffers logged since (notifyNewBufferAdded :262-277).  A gap makes the engine report
	 *  CLG_E_EPOCH_GAP, and next() throws the reference's NullPointerException there. */
	private final class LiveReplay extends InFlightLogIterator<Buffer> {
		private Chunk c;
		private int left;

		LiveReplay(Chunk first) {
			this.c = first;
			this.left = first.remaining;
		}

		/** The next chunk when this one is used up (buffers logged meanwhile included). */
		private void refill() {
			synchronized (EngineInFlightLog.this) {
				if (c.has() || c.status != CLG_OK) {
					return;
				}
				flush();
				Chunk n = fetch(0, 0, CLG_IFL_CONTINUE);
				left = n.remaining;
				c = n;
			}
		}

		@Override
		public boolean hasNext() { // consumerCursor.hasNext(): remaining > 0
			refill();
			return c.has() || c.status == CLG_E_EPOCH_GAP;
		}

		@Override
		public Buffer next() {
			refill();
			if (!c.has()) {
				check(c.status);
				throw new java.util.NoSuchElementException();
			}
			left--;
			return materialise(c, true);
		}

		@Override
		public Buffer peekNext() {
			refill();
			if (!c.has()) {
				check(c.status);
				throw new java.util.NoSuchElementException();
			}
			return materialise(c, false);
		}

		@Override
		public int numberRemaining() {
			return left;
		}

		@Override
		public long getEpoch() { // consumerCursor.getNextEpoch() :166-168
			refill();
			return c.epoch();
		}

		@Override
		public void close() { // :232-253: the rest is taken and recycled
			synchronized (EngineInFlightLog.this) {
				while (c.status == CLG_OK && (c.has() || left > 0)) {
					c.next = c.count;
					refill();
					if (!c.has()) {
						break;
					}
				}
			}
		}
	}
}
