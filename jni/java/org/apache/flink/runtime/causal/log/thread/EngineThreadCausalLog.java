/*
 * EngineThreadCausalLog -- drop-in ThreadCausalLog (ThreadCausalLog.java:33-96) whose
 * bytes live in MI355X HBM and whose metadata lives in the native engine, with the exact
 * semantics of ThreadCausalLogImpl (:51-527).  Construction replaces
 * `new ThreadCausalLogImpl(...)` at JobCausalLogImpl.java:136,162 and
 * AbstractDeltaSerializerDeserializer.java:171 (see INTEGRATION.md).
 *
 * Ownership follows the reference: getDeltaForConsumer / getDeterminants return a fresh
 * buffer the caller releases (Unpooled.EMPTY_BUFFER when empty, :265 / :287); the
 * upstream delta is copied during the call (Abstract...:155 slices are call-scoped).
 *
 * Source-only: this container has no JDK, so the binding is not compiled here.
 */
package org.apache.flink.runtime.causal.log.thread;

import org.apache.flink.runtime.causal.determinant.Determinant;
import org.apache.flink.runtime.causal.determinant.DeterminantEncoder;
import org.apache.flink.runtime.causal.engine.ClonosEngine;
import org.apache.flink.runtime.causal.log.job.CausalLogID;
import org.apache.flink.runtime.io.network.partition.consumer.InputChannelID;
import org.apache.flink.shaded.netty4.io.netty.buffer.ByteBuf;
import org.apache.flink.shaded.netty4.io.netty.buffer.ByteBufAllocator;
import org.apache.flink.shaded.netty4.io.netty.buffer.Unpooled;

import java.nio.ByteBuffer;

import static org.apache.flink.runtime.causal.engine.ClonosEngine.*;

public class EngineThreadCausalLog implements ThreadCausalLog {

	private final ClonosEngine engine;
	private final int log;
	private final CausalLogID causalLogID;
	private final DeterminantEncoder encoder;
	private final ByteBufAllocator alloc;
	// per-thread scratch for encoding one determinant (largest fixed record is 27 B)
	private final ThreadLocal<ByteBuf> scratch;

	public EngineThreadCausalLog(ClonosEngine engine, int job, CausalLogID id, DeterminantEncoder encoder,
								 ByteBufAllocator alloc) {
		this(engine, engine.openLog(job, id.getVertexID(), id.isMainThread(), id.getIntermediateDataSetLower(),
			id.getIntermediateDataSetUpper(), id.getSubpartitionIndex()), id, encoder, alloc);
	}

	/** A log the engine already opened (clg_process_delta's insertNewUpstreamLog,
	 *  AbstractDeltaSerializerDeserializer.java:165-194). */
	public static EngineThreadCausalLog wrap(ClonosEngine engine, int handle, CausalLogID id, DeterminantEncoder encoder,
											 ByteBufAllocator alloc) {
		return new EngineThreadCausalLog(engine, handle, id, encoder, alloc);
	}

	private EngineThreadCausalLog(ClonosEngine engine, int handle, CausalLogID id, DeterminantEncoder encoder,
								  ByteBufAllocator alloc) {
		this.engine = engine;
		this.causalLogID = id;
		this.encoder = encoder;
		this.alloc = alloc;
		this.log = handle;
		this.scratch = ThreadLocal.withInitial(() -> Unpooled.directBuffer(256));
	}

	@Override
	public CausalLogID getCausalLogID() {
		return causalLogID;
	}

	/** The engine handle of this log (batched natives take handles). */
	public int handle() {
		return log;
	}

	@Override
	public ByteBuf getDeterminants(long startEpochID) {
		int[] n = new int[1];
		int st = nGetDeterminants(engine.handle(), log, startEpochID, null, n);
		ByteBuf out = null;
		// an append may land between the size probe and the fetch (the task thread appends
		// while a Netty thread slices): CLG_E_CAPACITY reports the new size, nothing moved, retry
		while (st == CLG_E_CAPACITY) {
			if (out != null) {
				out.release();
			}
			int want = n[0] + SLACK;
			out = alloc.directBuffer(want);
			st = nGetDeterminants(engine.handle(), log, startEpochID, out.nioBuffer(0, want), n);
		}
		return finish(st, out, n[0]);
	}

	/** Extra room per fetch so a concurrent append rarely forces a second round. */
	private static final int SLACK = 256;

	private static ByteBuf finish(int st, ByteBuf out, int n) {
		if (st != CLG_OK) {
			if (out != null) {
				out.release();
			}
			check(st);
		}
		if (n == 0) {
			if (out != null) {
				out.release();
			}
			return Unpooled.EMPTY_BUFFER; // :265 / :287
		}
		return out.writerIndex(n);
	}

	@Override
	public int logLength() {
		int[] n = new int[1];
		check(nLogLength(engine.handle(), log, n));
		return n[0];
	}

	@Override
	public void processUpstreamDelta(ByteBuf delta, int offsetFromEpoch, long epochID) {
		ByteBuf direct = delta.isDirect() ? delta : Unpooled.directBuffer(delta.readableBytes()).writeBytes(delta.duplicate());
		try {
			ByteBuffer nio = direct.nioBuffer(direct.readerIndex(), direct.readableBytes());
			check(nUpstreamDelta(engine.handle(), log, epochID, offsetFromEpoch, nio, 0, nio.remaining()));
		} finally {
			if (direct != delta) {
				direct.release();
			}
		}
	}

	@Override
	public void appendDeterminant(Determinant determinant, long epochID) {
		ByteBuf buf = scratch.get().clear();
		encoder.encodeTo(determinant, buf); // SimpleDeterminantEncoder.encodeTo :56-75
		ByteBuffer nio = buf.nioBuffer(0, buf.writerIndex());
		int st;
		while ((st = nAppend(engine.handle(), log, epochID, nio, 0, nio.remaining())) == CLG_E_NOSPACE) {
			Thread.yield(); // mimics requestBufferBlocking (ThreadCausalLogImpl.java:444)
		}
		check(st);
	}

	@Override
	public boolean hasDeltaForConsumer(InputChannelID outputChannelID, long epochID) {
		int[] out = new int[1];
		check(nHasDelta(engine.handle(), log, outputChannelID.getLowerPart(), outputChannelID.getUpperPart(), epochID,
			out));
		return out[0] != 0;
	}

	@Override
	public int getOffsetFromEpochForConsumer(InputChannelID outputChannelID, long epochID) {
		int[] out = new int[1];
		check(nOffsetFromEpoch(engine.handle(), log, outputChannelID.getLowerPart(), outputChannelID.getUpperPart(),
			out));
		return out[0];
	}

	@Override
	public ByteBuf getDeltaForConsumer(InputChannelID outputChannelID, long epochID) {
		long lo = outputChannelID.getLowerPart(), hi = outputChannelID.getUpperPart();
		int[] n = new int[1];
		int st = nGetDelta(engine.handle(), log, lo, hi, epochID, null, n); // size probe, no advance
		ByteBuf out = null;
		// CLG_E_CAPACITY never advances the consumer, so a delta that grew since the probe
		// (a concurrent appendDeterminant) is fetched again at its new size
		while (st == CLG_E_CAPACITY) {
			if (out != null) {
				out.release();
			}
			int want = n[0] + SLACK;
			out = alloc.directBuffer(want);
			st = nGetDelta(engine.handle(), log, lo, hi, epochID, out.nioBuffer(0, want), n);
		}
		return finish(st, out, n[0]);
	}

	@Override
	public void notifyCheckpointComplete(long checkpointID) {
		check(nNotifyCheckpointComplete(engine.handle(), log, checkpointID));
	}

	@Override
	public void close() {
		check(nLogClose(engine.handle(), log));
	}

	@Override
	public void unregisterConsumer(InputChannelID toCancel) {
		check(nUnregisterConsumer(engine.handle(), log, toCancel.getLowerPart(), toCancel.getUpperPart()));
	}
}
