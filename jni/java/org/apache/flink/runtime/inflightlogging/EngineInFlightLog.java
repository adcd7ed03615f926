/*
 * InFlightLog over the MI355X engine (C-ABI clg_ifl_*, jni/clonos_jni.c): a drop-in for
 * InMemorySubpartitionInFlightLogger (InMemorySubpartitionInFlightLogger.java:28-207).
 * Buffer bytes are copied into HBM on log() and the Java Buffer is recycled at once; a
 * replay gathers every buffer from the start epoch in one GPU call and hands them out as
 * Buffers taken from the in-flight buffer pool.  Wiring: InMemoryInFlightLogFactory
 * returns `new EngineInFlightLog(engine)` instead of the in-memory logger.
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
	private BufferPool inFlightBufferPool;

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

	public EngineInFlightLog(ClonosEngine engine) {
		this.engine = engine;
		int[] h = new int[1];
		check(nIflOpen(engine.handle(), h));
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
			submit(new long[]{epochID}, new int[]{n}, direct, 1);
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
		submit(stagedEpochs, stagedLens, stage, staged);
		stage.clear();
		staged = 0;
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
	private void submit(long[] epochs, int[] lens, ByteBuffer bytes, int n) {
		submitting = true;
		try {
			int st;
			while ((st = nIflLogBatch(engine.handle(), ifl, epochs, lens, bytes, n)) == CLG_E_NOSPACE) {
				if (closed) {
					throw new IllegalStateException("in-flight log closed while waiting for pool space");
				}
				waitQuietly();
			}
			check(st);
		} finally {
			submitting = false;
			notifyAll();
		}
	}

	@Override
	public synchronized void notifyCheckpointComplete(long checkpointId) { // :51-70
		// free the pool first: a log() waiting for space (backpressure) can then finish
		check(nIflNotifyCheckpointComplete(engine.handle(), ifl, checkpointId));
		notifyAll();
		awaitNoSubmit();
		// staged buffers of truncated epochs never reach HBM, and a batch that was waiting
		// for space when this call began is truncated too: the reference truncates every
		// buffer logged before the notification
		dropStagedBelow(checkpointId);
		check(nIflNotifyCheckpointComplete(engine.handle(), ifl, checkpointId));
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
		long[] res = new long[7];
		int st = nIflReplay(engine.handle(), ifl, startEpochID, ignoreBuffers, null, null, null, res);
		if (st != CLG_OK && st != CLG_E_CAPACITY) {
			check(st);
		}
		ByteBuffer out = ByteBuffer.allocateDirect((int) Math.max(1, res[4]));
		ByteBuffer sizes = ByteBuffer.allocateDirect((int) Math.max(4, 4 * res[5])).order(ByteOrder.nativeOrder());
		ByteBuffer epochs = ByteBuffer.allocateDirect((int) Math.max(8, 8 * res[5])).order(ByteOrder.nativeOrder());
		check(nIflReplay(engine.handle(), ifl, startEpochID, ignoreBuffers, out, sizes, epochs, res));
		int status = (int) res[0];
		if (status != CLG_OK && status != CLG_E_EPOCH_GAP) { // the skip loop inside getInFlightIterator threw (:78-79)
			throw inFlightException(status, nLastError());
		}
		return new Replay(out, sizes, epochs, (int) res[1], (int) res[2], res[6], status);
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

	/** The drained ReplayIterator (:107-201): buffers materialised from the gathered bytes. */
	private final class Replay extends InFlightLogIterator<Buffer> {
		private final ByteBuffer bytes;
		private final ByteBuffer sizes;
		private final ByteBuffer epochs;
		private final int count;
		private final long endEpoch;
		private final int status;
		private int next;
		private int left;
		private int pos;

		Replay(ByteBuffer bytes, ByteBuffer sizes, ByteBuffer epochs, int count, int remaining, long endEpoch,
			int status) {
			this.bytes = bytes;
			this.sizes = sizes;
			this.epochs = epochs;
			this.count = count;
			this.left = remaining;
			this.endEpoch = endEpoch;
			this.status = status;
		}

		@Override
		public boolean hasNext() {
			// at a gap the reference still sees the last buffer before it (:146-149); next() throws (:156 -> :133)
			return next < count || status == CLG_E_EPOCH_GAP;
		}

		private Buffer materialise(boolean advance) {
			int n = sizes.getInt(4 * next);
			Buffer b;
			try {
				b = inFlightBufferPool.requestBufferBlocking();
			} catch (IOException | InterruptedException e) {
				throw new RuntimeException(e);
			}
			ByteBuffer src = bytes.duplicate();
			src.position(pos).limit(pos + n);
			b.getMemorySegment().put(0, src, n);
			b.setSize(n);
			if (advance) {
				pos += n;
				next++;
				left--;
			}
			return b;
		}

		@Override
		public Buffer next() {
			if (next >= count) {
				check(status); // CLG_E_EPOCH_GAP -> the reference's NullPointerException
				throw new java.util.NoSuchElementException();
			}
			return materialise(true);
		}

		@Override
		public Buffer peekNext() {
			if (next >= count) {
				throw new java.util.NoSuchElementException();
			}
			return materialise(false);
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
			return next < count ? epochs.getLong(8 * next) : endEpoch;
		}

		@Override
		public void close() {
			next = count;
		}
	}
}
