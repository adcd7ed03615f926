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
		ByteBuffer nio = buffer.getNioBufferReadable();
		int n = nio.remaining();
		if (n > stage.remaining() || staged == STAGE_BUFFERS) {
			flush();
		}
		if (n > STAGE_BYTES) { // larger than the stage: a batch of its own
			ByteBuffer direct = nio.isDirect() ? nio.slice() : ByteBuffer.allocateDirect(n).put(nio.duplicate());
			logBatch(new long[]{epochID}, new int[]{n}, direct, 1);
			return;
		}
		stage.put(nio.duplicate());
		stagedEpochs[staged] = epochID;
		stagedLens[staged] = n;
		staged++;
	}

	private void flush() {
		if (staged == 0) {
			return;
		}
		logBatch(stagedEpochs, stagedLens, stage, staged);
		stage.clear();
		staged = 0;
	}

	// Backpressure: a full in-flight pool (CLG_E_NOSPACE, nothing logged) waits until a
	// checkpoint completes and frees epochs (notifyCheckpointComplete wakes us), then retries.
	private void logBatch(long[] epochs, int[] lens, ByteBuffer bytes, int n) {
		int st;
		while ((st = nIflLogBatch(engine.handle(), ifl, epochs, lens, bytes, n)) == CLG_E_NOSPACE) {
			try {
				wait(10);
			} catch (InterruptedException e) {
				Thread.currentThread().interrupt();
				throw new RuntimeException(e);
			}
		}
		check(st);
	}

	@Override
	public synchronized void notifyCheckpointComplete(long checkpointId) { // :51-70
		flush();
		check(nIflNotifyCheckpointComplete(engine.handle(), ifl, checkpointId));
		notifyAll();
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
