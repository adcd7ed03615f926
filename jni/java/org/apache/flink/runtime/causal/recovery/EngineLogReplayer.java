/*
 * EngineLogReplayer -- drop-in for LogReplayerImpl (LogReplayerImpl.java:36-158): the main
 * thread's recovered log, replayed determinant by determinant.
 *
 * The only change is where the next determinant comes from: LogReplayerImpl.deserializeNext
 * (:138-145) calls determinantEncoder.decodeNext on the log, walking it byte by byte; here the
 * whole log is decoded once by the engine (EngineDecodedLog, clg_decode_host) and each
 * deserializeNext hands out the next record, materialised by the reference's own per-type
 * reader.  Replay order, DeterminantPool recycling, the async-event record-count checks
 * (:102-119), the finish check (:121-136) and the exceptions a malformed log raises are the
 * reference's: the engine stops at the first bad record and the reference's decodeNext
 * decodes it.
 *
 * ReplayingState (:67-69) swaps `new LogReplayerImpl(log, context)` for
 * `new EngineLogReplayer(log, context, engine)`.
 *
 * Source-only: this container has no JDK, so the binding is not compiled here.
 */
package org.apache.flink.runtime.causal.recovery;

import org.apache.flink.runtime.causal.determinant.AsyncDeterminant;
import org.apache.flink.runtime.causal.determinant.Determinant;
import org.apache.flink.runtime.causal.determinant.OrderDeterminant;
import org.apache.flink.runtime.causal.determinant.RNGDeterminant;
import org.apache.flink.runtime.causal.determinant.SerializableDeterminant;
import org.apache.flink.runtime.causal.determinant.TimestampDeterminant;
import org.apache.flink.runtime.causal.engine.ClonosEngine;
import org.apache.flink.runtime.causal.engine.EngineDecodedLog;
import org.apache.flink.runtime.causal.log.job.CausalLogID;
import org.apache.flink.shaded.netty4.io.netty.buffer.ByteBuf;
import org.slf4j.Logger;
import org.slf4j.LoggerFactory;

public class EngineLogReplayer implements LogReplayer {

	private static final Logger LOG = LoggerFactory.getLogger(LogReplayer.class);

	private final ByteBuf log;
	private final EngineDecodedLog decoded; // null when there is no log (nothing to replay)
	private final DeterminantPool determinantPool;
	private final RecoveryManagerContext context;

	Determinant nextDeterminant;

	private boolean done;

	public EngineLogReplayer(ByteBuf log, RecoveryManagerContext recoveryManagerContext, ClonosEngine engine) {
		this.context = recoveryManagerContext;
		this.log = log;
		this.decoded = log == null ? null
			: new EngineDecodedLog(engine, log, context.causalLog.getDeterminantEncoder());
		this.determinantPool = new DeterminantPool();
		deserializeNext();
		done = false;
	}

	@Override
	public synchronized int replayRandomInt() {
		assert nextDeterminant instanceof RNGDeterminant;
		final RNGDeterminant d = (RNGDeterminant) nextDeterminant;
		deserializeNext();
		int toReturn = d.getNumber();
		postHook(d);
		return toReturn;
	}

	@Override
	public synchronized byte replayNextChannel() {
		assert nextDeterminant instanceof OrderDeterminant;
		final OrderDeterminant d = (OrderDeterminant) nextDeterminant;
		deserializeNext();
		byte toReturn = d.getChannel();
		postHook(d);
		return toReturn;
	}

	@Override
	public synchronized long replayNextTimestamp() {
		assert nextDeterminant instanceof TimestampDeterminant;
		final TimestampDeterminant d = (TimestampDeterminant) nextDeterminant;
		deserializeNext();
		long toReturn = d.getTimestamp();
		postHook(d);
		return toReturn;
	}

	@Override
	public synchronized Object replaySerializableDeterminant() {
		assert nextDeterminant instanceof SerializableDeterminant;
		final SerializableDeterminant d = (SerializableDeterminant) nextDeterminant;
		deserializeNext();
		Object toReturn = d.getDeterminant();
		postHook(d);
		return toReturn;
	}

	@Override
	public synchronized void triggerAsyncEvent() {
		assert nextDeterminant instanceof AsyncDeterminant;
		AsyncDeterminant asyncDeterminant = (AsyncDeterminant) nextDeterminant;
		int currentRecordCount = context.epochTracker.getRecordCount();
		if (LOG.isDebugEnabled())
			LOG.debug("Trigger {}", asyncDeterminant);
		if (currentRecordCount != asyncDeterminant.getRecordCount())
			throw new RuntimeException("Current record count is not the determinants record count. Current: "
				+ currentRecordCount + ", determinant: " + asyncDeterminant.getRecordCount());
		// the callback may itself replay a determinant: advance first, as the reference does
		deserializeNext();
		asyncDeterminant.process(context);
		postHook(asyncDeterminant);
	}

	public synchronized void checkFinished() {
		if (!done && nextDeterminant == null) {
			if (log != null) {
				done = true;
				assert log.capacity() ==
					context.causalLog.threadLogLength(new CausalLogID(context.getTaskVertexID()));
				log.release();
			}
			LOG.info("Finished recovering main thread! Transitioning to RunningState!");
			context.owner.setState(new RunningState(context.owner, context));
		}
	}

	private void deserializeNext() {
		nextDeterminant = null;
		if (decoded != null && log.isReadable()) {
			nextDeterminant = decoded.next(determinantPool);
			if (LOG.isDebugEnabled())
				LOG.debug("Deserialized nextDeterminant: {}", nextDeterminant);
		}
	}

	private void postHook(Determinant determinant) {
		determinantPool.recycle(determinant);
		if (nextDeterminant instanceof AsyncDeterminant)
			context.epochTracker.setRecordCountTarget(((AsyncDeterminant) nextDeterminant).getRecordCount());
		checkFinished();
	}
}
